#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/dbg; mkdir -p $O
S=scripts/gpu_step.sh
$S 120 $O/fill.log python -u scripts/debug_fill.py
cat $O/fill.log
$S 300 $O/golden.log python -u -m pytest tests/test_gpu_golden.py -q --timeout 300 --timeout-method thread
tail -5 $O/golden.log
