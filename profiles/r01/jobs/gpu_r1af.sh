#!/bin/bash
# Chained vs independent temporal tiles, same state sequence per mode.
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1af; mkdir -p $O
S=$R/scripts/gpu_step.sh
$S 300 $O/chain_sweep.log python -u scripts/chain_sweep.py
cat $O/chain_sweep.log
