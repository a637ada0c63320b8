#!/bin/bash
# DPP row-rotate neighbours in the windowed small-grid kernel: small-grid parity + golden, then the deep sweep.
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1ak; mkdir -p $O
S=$R/scripts/gpu_step.sh
$S 400 $O/pytest_small.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -m gpu -x -q -k "small or golden or p46 or cfg" --timeout 120 --timeout-method thread
tail -5 $O/pytest_small.log
$S 300 $O/p46_window_deep.log python -u scripts/p46_window.py deep
cat $O/p46_window_deep.log
