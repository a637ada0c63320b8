#!/bin/bash
# r2j: runtime ghost depth for the tiles; generations per launch 12..32 at
# 65536^2 bit / byte, the driver's 20-step shape, 32768^2; then the GPU suite
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2j
mkdir -p $O
S=scripts/gpu_step.sh
B="python -u bench.py --no-cpu-baseline"
for round in 1 2; do
  for bg in 12 16 20 24 32; do
    $S 120 $O/bit_b${bg}_$round.json env LIFE_BLOCK_GENS=$bg $B --steps 480 --warmup 48 || exit $?
  done
done
for bg in 16 24 32; do
  $S 120 $O/byte_b${bg}.json env LIFE_BLOCK_GENS=$bg $B --kernel byte --steps 480 --warmup 48 || exit $?
  $S 120 $O/bit32768_b${bg}.json env LIFE_BLOCK_GENS=$bg $B --size 32768 --steps 480 --warmup 48 || exit $?
  $S 120 $O/byte32768_b${bg}.json env LIFE_BLOCK_GENS=$bg $B --kernel byte --size 32768 --steps 480 --warmup 48 || exit $?
done
for bg in 16 20 32; do
  $S 120 $O/driver_b${bg}.json env LIFE_BLOCK_GENS=$bg $B --steps 20 --warmup 5 || exit $?
done
$S 1200 $O/pytest.log python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread
