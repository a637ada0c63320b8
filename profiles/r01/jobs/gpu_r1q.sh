#!/bin/bash
# hsum mode 2 (DPP left + ds_bpermute right) as default: parity, rows sweep both encodings.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r1q; mkdir -p $O
S=scripts/gpu_step.sh
$S 400 $O/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread
tail -2 $O/pytest_gpu.log
$S 240 $O/tune_bit.log python -u scripts/tune.py --kernels bit --temporal 32,48,64,80,96 --gens 2
$S 240 $O/tune_byte.log python -u scripts/tune.py --kernels byte --temporal 32,48,64,80,96 --gens 2
grep -h '^{' $O/tune_*.log | cut -c1-200
