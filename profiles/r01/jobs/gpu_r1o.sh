#!/bin/bash
# Census/checksum + full-size parity (C3-C5), then the whole GPU suite.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r1o; mkdir -p $O
S=scripts/gpu_step.sh
$S 600 $O/pytest_fullsize.log python -u -m pytest tests/test_gpu_fullsize.py -v --timeout 180 --timeout-method thread --durations=0
grep -E "PASS|FAIL|ERROR|passed|failed|s call" $O/pytest_fullsize.log | tail -40
$S 400 $O/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread
tail -3 $O/pytest_gpu.log
