#!/bin/bash
# configs[1] p46gun_big: small LDS kernel vs temporal tiles (K 32 / 16).
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1y; mkdir -p $O
S=$R/scripts/gpu_step.sh
$S 200 $O/p46_k32.log python -u scripts/p46_modes.py
cat $O/p46_k32.log
LIFE_TEMPORAL_DEPTH=16 $S 200 $O/p46_k16.log python -u scripts/p46_modes.py
cat $O/p46_k16.log
