#!/bin/bash
# r04ah: confirmation after the fast-wrap margin change: smoke, the whole GPU
# suite, the driver-shaped bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04/ah; mkdir -p $O
S=scripts/gpu_step.sh
$S 120 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
$S 900 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
$S 200 $O/bench_driver.log python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
echo done
