#!/bin/bash
# Tile height x K sweep (hsum mode 2): bit rows 40-64, byte rows 32-48, K 24/32.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r1r; mkdir -p $O
S=scripts/gpu_step.sh
$S 240 $O/bit_k32.log python -u scripts/tune.py --kernels bit --temporal 40,48,56,64 --gens 2
LIFE_TEMPORAL_DEPTH=24 $S 240 $O/bit_k24.log python -u scripts/tune.py --kernels bit --temporal 40,48,56,64 --gens 3
$S 240 $O/byte_k32.log python -u scripts/tune.py --kernels byte --temporal 32,40,48,56 --gens 2
LIFE_TEMPORAL_DEPTH_BYTE=24 $S 240 $O/byte_k24.log python -u scripts/tune.py --kernels byte --temporal 32,40,48 --gens 3
for f in $O/*.log; do echo "== $f"; grep -h '^{' $f | cut -c1-170; done
