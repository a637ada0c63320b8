#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2h
mkdir -p $O
scripts/gpu_step.sh 1200 $O/pytest.log python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread
