#!/bin/bash
# r2k: byte tiles A/B, previous commit (ghost depth = template K) vs runtime ghost depth
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2k
mkdir -p $O
S=scripts/gpu_step.sh
B="python -u bench.py --no-cpu-baseline --kernel byte --steps 320 --warmup 32"
for round in 1 2; do
  $S 120 $O/prev_$round.json env LIFE_MI355X_LIB=build_exp/prev/liblife_mi355x.so $B || exit $?
  $S 120 $O/cur_$round.json env LIFE_BLOCK_GENS=32 $B || exit $?
done
