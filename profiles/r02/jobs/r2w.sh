#!/bin/bash
# r2w: banded last tile column (LIFE_BANDS) and 12-wave bit tiles (LIFE_TILE_WAVES=12): parity of the tile paths under
# both, A/B bench lines, kernel trace (VGPRs)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2w
mkdir -p $O
S=scripts/gpu_step.sh
R=$GRAFT_REPO_ROOT
$S 300 $O/pytest_bands.log python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "flow or temporal or timing or multi_shard or single_shard" || exit $?
grep -q " passed" $O/pytest_bands.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest_bands.log || exit 1
$S 300 $O/pytest12.log env LIFE_TILE_WAVES=12 python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread -k "flow or temporal or timing or multi_shard" || exit $?
grep -q " passed" $O/pytest12.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest12.log || exit 1
for round in 1 2; do
  for cfg in "8 0" "8 1" "12 1"; do
    set -- $cfg
    t=w$1_b$2
    $S 200 $O/${t}_65536_$round.json env LIFE_TILE_WAVES=$1 LIFE_BANDS=$2 python -u bench.py --no-cpu-baseline --steps 480 --warmup 32 || exit $?
    $S 200 $O/${t}_32768_$round.json env LIFE_TILE_WAVES=$1 LIFE_BANDS=$2 python -u bench.py --no-cpu-baseline --size 32768 --steps 480 --warmup 32 || exit $?
    $S 200 $O/${t}_driver_$round.json env LIFE_TILE_WAVES=$1 LIFE_BANDS=$2 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 || exit $?
  done
done
$S 200 $O/rocprof12.log env LIFE_TILE_WAVES=12 rocprofv3 --kernel-trace --stats -d $O/prof12 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 100 --warmup 20 || exit $?
$S 200 $O/rocprof8.log rocprofv3 --kernel-trace --stats -d $O/prof8 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --steps 100 --warmup 20 || exit $?
