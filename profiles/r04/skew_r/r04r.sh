#!/bin/bash
# r04r: skewed segments -- per-tile timelines at segment lengths 1/2/8 and
# with the issue priority falling as a segment progresses (LIFE_SKEW_PRIO).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04/r; mkdir -p $O
S=scripts/gpu_step.sh
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline"
for seg in 1 2 8; do
  LIFE_MI355X_LIB=build_exp/tr3/liblife_mi355x.so LIFE_SKEW=1 LIFE_SKEW_SEG=$seg $S 120 $O/trace_seg$seg.log python -u scripts/wg_trace.py 20 $O/trace_seg$seg.npy || exit $?
done
LIFE_MI355X_LIB=build_exp/tp3/liblife_mi355x.so LIFE_SKEW=1 $S 120 $O/trace_prio.log python -u scripts/wg_trace.py 20 $O/trace_prio.npy || exit $?
LIFE_MI355X_LIB=build_exp/p3/liblife_mi355x.so LIFE_SKEW=1 $S 120 $O/test_p3.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k skew || exit $?
for i in 1 2; do
  LIFE_SKEW=0 $S 150 $O/base_$i.log $B || exit $?
  LIFE_MI355X_LIB=build_exp/p3/liblife_mi355x.so LIFE_SKEW=1 $S 150 $O/p3_$i.log $B || exit $?
done
echo done
