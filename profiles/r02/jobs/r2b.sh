#!/bin/bash
# r2b: sweep kernel with buffer-resource loads/stores -- parity suite, then A/B
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2b
mkdir -p $O
S=scripts/gpu_step.sh
$S 900 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread || exit $?
B="python -u bench.py --no-cpu-baseline"
$S 180 $O/bit_sweep16.json $B --steps 320 --warmup 32 || exit $?
$S 180 $O/bit_sweep12.json env LIFE_TEMPORAL_DEPTH=12 $B --steps 324 --warmup 36 || exit $?
$S 180 $O/bit_sweep8.json env LIFE_TEMPORAL_DEPTH=8 $B --steps 320 --warmup 32 || exit $?
$S 180 $O/bit_sweep16_w2048.json env LIFE_SWEEP_WAVES=2048 $B --steps 320 --warmup 32 || exit $?
$S 180 $O/bit_sweep12_w2048.json env LIFE_SWEEP_WAVES=2048 LIFE_TEMPORAL_DEPTH=12 $B --steps 324 --warmup 36 || exit $?
$S 180 $O/bit_tiles32.json env LIFE_TEMPORAL_DEPTH=32 $B --temporal tiles --steps 320 --warmup 32 || exit $?
$S 180 $O/byte_sweep16.json env LIFE_TEMPORAL_DEPTH_BYTE=16 $B --kernel byte --steps 320 --warmup 32 || exit $?
$S 180 $O/bit_sweep16_32768.json $B --size 32768 --steps 320 --warmup 32 || exit $?
$S 180 $O/bit_sweep16_driver.json $B --steps 20 --warmup 5 || exit $?
