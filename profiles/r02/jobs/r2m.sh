#!/bin/bash
# r2m: tile height R x generations per launch m at 32768^2 and 65536^2 (bit), byte R at both sizes
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2m
mkdir -p $O
S=scripts/gpu_step.sh
B="python -u bench.py --no-cpu-baseline --steps 480 --warmup 48"
for size in 32768 65536; do
  for R in 32 40 48 56 64; do
    for m in 16 20 32; do
      $S 120 $O/bit_${size}_R${R}_m${m}.json env LIFE_TEMPORAL_ROWS=$R LIFE_BLOCK_GENS=$m $B --size $size || exit $?
    done
  done
  for R in 32 40 48; do
    $S 120 $O/byte_${size}_R${R}.json env LIFE_TEMPORAL_ROWS_BYTE=$R $B --kernel byte --size $size || exit $?
  done
done
