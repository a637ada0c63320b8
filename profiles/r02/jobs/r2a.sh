#!/bin/bash
# r2a: first sweep-kernel run -- GPU parity suite, then 65536^2 bench A/B
# (sweep K = 8/12/16 vs the round-1 tiles at K = 32), byte, 32768^2, and the
# driver's --steps 20 --warmup 5 shape.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2a
mkdir -p $O
S=scripts/gpu_step.sh
$S 900 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread || exit $?
B="python -u bench.py --no-cpu-baseline"
$S 180 $O/bit_sweep16.json $B --steps 320 --warmup 32 || exit $?
$S 180 $O/bit_sweep12.json env LIFE_TEMPORAL_DEPTH=12 $B --steps 324 --warmup 36 || exit $?
$S 180 $O/bit_sweep8.json env LIFE_TEMPORAL_DEPTH=8 $B --steps 320 --warmup 32 || exit $?
$S 180 $O/bit_tiles32.json env LIFE_TEMPORAL_DEPTH=32 $B --temporal tiles --steps 320 --warmup 32 || exit $?
$S 180 $O/byte_sweep.json $B --kernel byte --steps 320 --warmup 32 || exit $?
$S 180 $O/byte_tiles.json $B --kernel byte --temporal tiles --steps 320 --warmup 32 || exit $?
$S 180 $O/bit_sweep16_32768.json $B --size 32768 --steps 320 --warmup 32 || exit $?
$S 180 $O/bit_tiles32_32768.json env LIFE_TEMPORAL_DEPTH=32 $B --size 32768 --temporal tiles --steps 320 --warmup 32 || exit $?
$S 180 $O/bit_sweep16_driver.json $B --steps 20 --warmup 5 || exit $?
$S 180 $O/bit_tiles32_driver.json env LIFE_TEMPORAL_DEPTH=32 $B --temporal tiles --steps 20 --warmup 5 || exit $?
