#!/bin/bash
# r06j: the random-shape tail-split test (new), then smoke and the whole GPU
# suite on the final library.  Expectation: all green.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/j; mkdir -p $O
S=scripts/gpu_step.sh
T="python -u -m pytest -x -q --timeout 600 --timeout-method thread -p no:cacheprovider"
$S 300 $O/pytest_new.log $T tests/test_gpu_fullsize.py -m gpu -k "random_shapes" -v || exit $?
grep -q " passed" $O/pytest_new.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest_new.log || exit 1
$S 120 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
$S 200 $O/bench_driver.log python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
$S 1000 $O/pytest.log $T tests -m gpu || exit $?
grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
echo done
