#!/bin/bash
# r04t: skewed segments dealt XCD-aware (a segment row's tile columns on one
# L2), with and without the falling priority; HBM fetch of the best.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r04/t; mkdir -p $O
S=scripts/gpu_step.sh
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline"
for v in x3 xp3; do
  LIFE_MI355X_LIB=build_exp/$v/liblife_mi355x.so LIFE_SKEW=1 $S 120 $O/test_$v.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k skew || exit $?
done
for i in 1 2; do
  LIFE_SKEW=0 $S 150 $O/base_$i.log $B || exit $?
  for v in x3 xp3; do LIFE_MI355X_LIB=build_exp/$v/liblife_mi355x.so LIFE_SKEW=1 $S 150 $O/${v}_$i.log $B || exit $?; done
done
LIFE_MI355X_LIB=build_exp/txp3/liblife_mi355x.so LIFE_SKEW=1 $S 120 $O/trace_xp3.log python -u scripts/wg_trace.py 20 $O/trace_xp3.npy || exit $?
cd /tmp && export TMPDIR=/tmp && cd $R
for v in x3 xp3; do
  LIFE_MI355X_LIB=$R/build_exp/$v/liblife_mi355x.so LIFE_SKEW=1 $S 90 $O/pmc_$v.log timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_$v -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
done
echo done
