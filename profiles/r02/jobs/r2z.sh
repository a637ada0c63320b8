#!/bin/bash
# r2z: half-height tail tiles for one-launch step calls (LIFE_TAIL_SPLIT, bit and byte) + banded column: parity,
# A/B vs the previous commit's library and with the split off
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2z
mkdir -p $O
S=scripts/gpu_step.sh
$S 400 $O/pytest_tiles.log python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -k "flow or temporal or timing or multi_shard or single_shard or c4 or c3 or split" || exit $?
grep -q " passed" $O/pytest_tiles.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest_tiles.log || exit 1
B=$GRAFT_REPO_ROOT/build_exp/base/liblife_mi355x.so
for round in 1 2; do
  for v in base s0 s1; do
    case $v in base) E="LIFE_MI355X_LIB=$B";; s0) E="LIFE_TAIL_SPLIT=0";; s1) E="LIFE_TAIL_SPLIT=1";; esac
    $S 200 $O/${v}_driver_$round.json env $E python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 || exit $?
    $S 200 $O/${v}_32768_byte_$round.json env $E python -u bench.py --no-cpu-baseline --size 32768 --kernel byte --steps 480 --warmup 32 || exit $?
    $S 200 $O/${v}_32768_driver_$round.json env $E python -u bench.py --no-cpu-baseline --size 32768 --steps 20 --warmup 5 || exit $?
  done
done
