#!/bin/bash
# r2g: sweep (DPP left word) at 12 / 16 stages vs tiles at K = 16 / 32; bit 65536^2
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2g
mkdir -p $O
S=scripts/gpu_step.sh
B="python -u bench.py --no-cpu-baseline --steps 192 --warmup 48"
D=build_exp/dpp/liblife_mi355x.so
for round in 1 2; do
  $S 120 $O/dpp16_$round.json env LIFE_MI355X_LIB=$D $B || exit $?
  $S 120 $O/dpp12_$round.json env LIFE_MI355X_LIB=$D LIFE_TEMPORAL_DEPTH=12 $B || exit $?
  $S 120 $O/dpp12w4096_$round.json env LIFE_MI355X_LIB=$D LIFE_TEMPORAL_DEPTH=12 LIFE_SWEEP_WAVES=4096 $B || exit $?
  $S 120 $O/tiles16_$round.json $B --temporal tiles || exit $?
  $S 120 $O/tiles32_$round.json env LIFE_TEMPORAL_DEPTH=32 $B --temporal tiles || exit $?
done
