#!/bin/bash
# r3c: banded last column for the byte tiles too: tile-path parity (both encodings), A/B bands on/off
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3c
mkdir -p $O
S=scripts/gpu_step.sh
$S 400 $O/pytest_tiles.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_golden.py tests/test_gpu_loopback.py -m gpu -x -q --timeout 200 --timeout-method thread -k "temporal or timing or multi_shard or single_shard or split or c4 or c3 or byte or loopback" || exit $?
grep -q " passed" $O/pytest_tiles.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest_tiles.log || exit 1
for round in 1 2; do
  for b in 0 1; do
    $S 200 $O/byte_b${b}_$round.json env LIFE_BANDS=$b python -u bench.py --no-cpu-baseline --kernel byte --steps 480 --warmup 32 || exit $?
    $S 200 $O/byte_driver_b${b}_$round.json env LIFE_BANDS=$b python -u bench.py --no-cpu-baseline --kernel byte --steps 20 --warmup 5 || exit $?
  done
done
