#!/bin/bash
# r05y2: smoke, dataflow + golden tests and two lines on the final build (the
# timing-only dataflow switches removed after r05y: same code at their
# default).  Expectation: green, 32768^2 ~97 T, driver ~100 T.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/y2; mkdir -p $O
S=scripts/gpu_step.sh
$S 120 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
$S 600 $O/test_flow.log python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
$S 150 $O/c2_32768.log python -u bench.py --no-cpu-baseline --shape 32768x32768 || exit $?
$S 150 $O/bench_driver.log python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
echo done
