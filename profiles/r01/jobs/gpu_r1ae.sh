#!/bin/bash
# Chained temporal tiles: parity (temporal single/multi-shard, timing, full size), then A/B timing.
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1ae; mkdir -p $O
S=$R/scripts/gpu_step.sh
$S 300 $O/pytest_temporal.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "temporal or timing" --timeout 120 --timeout-method thread
tail -3 $O/pytest_temporal.log
$S 300 $O/pytest_full.log python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q --timeout 240 --timeout-method thread
tail -3 $O/pytest_full.log
$S 200 $O/chain_sweep.log python -u scripts/chain_sweep.py
cat $O/chain_sweep.log
