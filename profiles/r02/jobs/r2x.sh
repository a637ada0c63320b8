#!/bin/bash
# r2x: banded last tile column, compile-time instance: parity of the tile paths; A/B in one job against the previous
# commit's library (build_exp/base via LIFE_MI355X_LIB) with bands on / off
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2x
mkdir -p $O
S=scripts/gpu_step.sh
$S 300 $O/pytest_bands.log python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "flow or temporal or timing or multi_shard or single_shard" || exit $?
grep -q " passed" $O/pytest_bands.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest_bands.log || exit 1
B=$GRAFT_REPO_ROOT/build_exp/base/liblife_mi355x.so
for round in 1 2; do
  for v in base b0 b1; do
    case $v in base) E="LIFE_MI355X_LIB=$B";; b0) E="LIFE_BANDS=0";; b1) E="LIFE_BANDS=1";; esac
    $S 200 $O/${v}_driver_$round.json env $E python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 || exit $?
    $S 200 $O/${v}_65536_$round.json env $E python -u bench.py --no-cpu-baseline --steps 480 --warmup 32 || exit $?
    $S 200 $O/${v}_16384_$round.json env $E python -u bench.py --no-cpu-baseline --size 16384 --steps 960 --warmup 32 || exit $?
  done
done
