#!/bin/bash
# Window option validation + small-grid parity.
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1av; mkdir -p $O
S=$R/scripts/gpu_step.sh
$S 300 $O/pytest_small.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "small" --timeout 120 --timeout-method thread
tail -3 $O/pytest_small.log
