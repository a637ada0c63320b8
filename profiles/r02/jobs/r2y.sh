#!/bin/bash
# r2y: banded column in the per-launch tiles only (dataflow form restored): parity of the tile paths, A/B vs the
# previous commit's library
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2y
mkdir -p $O
S=scripts/gpu_step.sh
$S 300 $O/pytest_tiles.log python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 200 --timeout-method thread -k "flow or temporal or timing or multi_shard or single_shard or C4 or c4 or split" || exit $?
grep -q " passed" $O/pytest_tiles.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest_tiles.log || exit 1
B=$GRAFT_REPO_ROOT/build_exp/base/liblife_mi355x.so
for round in 1 2; do
  for v in base cur; do
    case $v in base) E="LIFE_MI355X_LIB=$B";; cur) E="LIFE_BANDS=1";; esac
    $S 200 $O/${v}_driver_$round.json env $E python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 || exit $?
    $S 200 $O/${v}_65536_$round.json env $E python -u bench.py --no-cpu-baseline --steps 480 --warmup 32 || exit $?
    $S 200 $O/${v}_loop_$round.json env $E python -u bench.py --no-cpu-baseline --steps 480 --warmup 32 --loopback || exit $?
  done
done
