#!/bin/bash
# Row-schedule experiments on the temporal kernel (bit, K=32): neighbour words
# via ds_bpermute, 16- and 4-wave tiles, vs the shipped build.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r1p; mkdir -p $O
S=scripts/gpu_step.sh
$S 200 $O/base.log python -u scripts/tune.py --kernels bit --temporal 48,80,96 --gens 2
for v in hsum1 hsum2; do
  LIFE_MI355X_LIB=$PWD/build_exp/$v/liblife_mi355x.so $S 200 $O/$v.log python -u scripts/tune.py --kernels bit --temporal 48,80,96 --gens 2
done
LIFE_MI355X_LIB=$PWD/build_exp/nw16/liblife_mi355x.so $S 200 $O/nw16.log python -u scripts/tune.py --kernels bit --temporal 32,48,64 --gens 2
LIFE_MI355X_LIB=$PWD/build_exp/nw4/liblife_mi355x.so $S 200 $O/nw4.log python -u scripts/tune.py --kernels bit --temporal 64,96 --gens 2
grep -h '^{' $O/*.log | cut -c1-200
