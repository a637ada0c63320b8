#!/bin/bash
# r5t: validation at HEAD (after the serial-schedule option): smoke, the whole GPU suite, the driver-
# shaped and default bench lines.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5t
mkdir -p $O
S=scripts/gpu_step.sh
$S 300 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
grep -q "smoke ok" $O/smoke.log || exit 1
$S 900 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
tail -2 $O/pytest.log; grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
$S 300 $O/bench_driver.json python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
$S 300 $O/bench_default.json python -u bench.py --no-cpu-baseline || exit $?
echo done
