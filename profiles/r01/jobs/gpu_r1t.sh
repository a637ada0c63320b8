#!/bin/bash
# XCD-aware tile order (column-major runs per XCD) vs default, both encodings.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r1t; mkdir -p $O
S=scripts/gpu_step.sh
$S 200 $O/base_bit.log python -u scripts/tune.py --kernels bit --temporal 48 --gens 2 --rounds 5
LIFE_MI355X_LIB=$PWD/build_exp/xcd/liblife_mi355x.so $S 200 $O/xcd_bit.log python -u scripts/tune.py --kernels bit --temporal 48 --gens 2 --rounds 5
$S 200 $O/base_byte.log python -u scripts/tune.py --kernels byte --temporal 32,48 --gens 2 --rounds 3
LIFE_MI355X_LIB=$PWD/build_exp/xcd/liblife_mi355x.so $S 200 $O/xcd_byte.log python -u scripts/tune.py --kernels byte --temporal 32,48 --gens 2 --rounds 3
for f in $O/*.log; do echo "== $f"; grep -h '^{' $f | cut -c1-170; done
