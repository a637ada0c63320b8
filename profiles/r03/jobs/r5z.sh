#!/bin/bash
# r5z: 32768^2 (configs[2]; 2.2 rounds of tiles per launch, so the per-launch ramp and tail weigh
# more than at 65536^2): generations per launch x tile shape on the default run.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5z
rm -rf $O; mkdir -p $O
S=scripts/gpu_step.sh
for i in 1 2; do
  for v in "12 24 8" "16 24 8" "20 24 8" "24 24 8" "12 16 8" "16 16 8" "20 24 12" "16 16 16"; do
    set -- $v
    LIFE_BLOCK_GENS=$1 LIFE_TEMPORAL_ROWS=$2 LIFE_TILE_WAVES=$3 $S 200 $O/s32k_m$1_$2x$3_$i.json python -u bench.py --size 32768 --no-cpu-baseline || exit $?
  done
done
echo done
