#!/bin/bash
# r2f: sweep-kernel variants A/B (bit 65536^2, K = 16): stage interleaving,
# DPP left word, occupancy target; two interleaved rounds
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2f
mkdir -p $O
S=scripts/gpu_step.sh
for round in 1 2; do
  for v in g1 g2 g4 dpp dppg2 g2o2 g4o2; do
    $S 120 $O/${v}_$round.json env LIFE_MI355X_LIB=build_exp/$v/liblife_mi355x.so python -u bench.py --no-cpu-baseline --steps 160 --warmup 16 || exit $?
  done
done
