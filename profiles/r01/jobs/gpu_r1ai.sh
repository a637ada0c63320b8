#!/bin/bash
# Windowed small-grid kernel: deep-halo sweep on p46gun_big.
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1ai; mkdir -p $O
S=$R/scripts/gpu_step.sh
$S 300 $O/p46_window_deep.log python -u scripts/p46_window.py deep
cat $O/p46_window_deep.log
