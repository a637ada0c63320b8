#!/bin/bash
# r5i: 63-pair tile columns (half-pair tile edges) on an x axis that wraps inside the shard:
# parity suites, then A/B LIFE_HALF_PAIRS 0/1 at the driver's shape, the default run and 32768^2.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5i
mkdir -p $O
S=scripts/gpu_step.sh
$S 700 $O/pytest.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py tests/test_gpu_flow.py tests/test_gpu_loopback.py -x -q --timeout 250 --timeout-method thread -p no:cacheprovider || exit $?
tail -2 $O/pytest.log; grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
for i in 1 2 3; do
  for h in 0 1; do
    LIFE_HALF_PAIRS=$h $S 200 $O/drv_h${h}_$i.json python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  done
done
for i in 1 2; do
  for h in 0 1; do
    LIFE_HALF_PAIRS=$h $S 200 $O/def_h${h}_$i.json python -u bench.py --no-cpu-baseline || exit $?
    LIFE_HALF_PAIRS=$h $S 200 $O/s32768_h${h}_$i.json python -u bench.py --size 32768 --no-cpu-baseline || exit $?
  done
done
echo done
