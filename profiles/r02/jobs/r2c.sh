#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2c
mkdir -p $O
timeout -k 10 300 python -u scripts/sweep_diag.py > $O/diag.log 2>&1 || exit $?
LIFE_TEMPORAL_DEPTH_BYTE=16 timeout -k 10 300 python -u scripts/sweep_diag.py > $O/diag_b16.log 2>&1
