#!/bin/bash
# r05y: final validation of the round-5 product after the dataflow warm-up
# (r05v): smoke, the whole GPU suite, the driver / default / configs[2] lines
# and rocprofv3 kernel stats of configs[2].  Expectation: all green; driver
# ~100 T, defaults ~112 T, 32768^2 ~97 T.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/y; mkdir -p $O
S=scripts/gpu_step.sh
$S 120 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
$S 200 $O/bench_driver.log python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
$S 200 $O/bench_default.log python -u bench.py --no-cpu-baseline || exit $?
$S 150 $O/c2_32768.log python -u bench.py --no-cpu-baseline --shape 32768x32768 || exit $?
$S 1100 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
echo done
