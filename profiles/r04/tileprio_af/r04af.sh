#!/bin/bash
# r04af: per-launch tiles with issue priority falling as a tile advances
# (LIFE_TILE_PRIO=1: the last-dispatched tiles catch up, the launch's tail
# shortens?) against the in-tree build; timelines of both.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04/af; mkdir -p $O
S=scripts/gpu_step.sh
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline"
L=build_exp/tp/liblife_mi355x.so
LIFE_MI355X_LIB=$L $S 300 $O/test_tp.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "bit and not skew" || exit $?
LIFE_MI355X_LIB=build_exp/trc/liblife_mi355x.so $S 120 $O/trace_base.log python -u scripts/wg_trace.py 20 $O/trace_base.npy || exit $?
LIFE_MI355X_LIB=build_exp/ttp/liblife_mi355x.so $S 120 $O/trace_tp.log python -u scripts/wg_trace.py 20 $O/trace_tp.npy || exit $?
for i in 1 2 3; do
  $S 150 $O/base_$i.log $B || exit $?
  LIFE_MI355X_LIB=$L $S 150 $O/tp_$i.log $B || exit $?
done
echo done
