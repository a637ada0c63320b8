#!/bin/bash
# Windowed small-grid kernel: parity (new + existing small-grid cases + golden), then the p46 sweep.
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1ah; mkdir -p $O
S=$R/scripts/gpu_step.sh
$S 400 $O/pytest_small.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -m gpu -x -q -k "small or golden or p46 or cfg" --timeout 120 --timeout-method thread
tail -5 $O/pytest_small.log
$S 300 $O/p46_window.log python -u scripts/p46_window.py
cat $O/p46_window.log
