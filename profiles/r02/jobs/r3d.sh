#!/bin/bash
# r3d: clock state vs soup for the driver-shaped call (scripts/preheat_probe.py)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3d
mkdir -p $O
scripts/gpu_step.sh 300 $O/preheat.jsonl python -u scripts/preheat_probe.py || exit $?
