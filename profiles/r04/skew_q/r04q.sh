#!/bin/bash
# r04q: skewed tiles, fence 3 (barrier pinned, rows above and their
# neighbours fetched right after it) and per-workgroup timelines of one
# launch of each kernel (diagnostics build).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04/q; mkdir -p $O
S=scripts/gpu_step.sh
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline"
LIFE_MI355X_LIB=build_exp/f3/liblife_mi355x.so LIFE_SKEW=1 $S 120 $O/test_f3.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k skew || exit $?
LIFE_MI355X_LIB=build_exp/tr3/liblife_mi355x.so LIFE_SKEW=0 $S 120 $O/trace_s0.log python -u scripts/wg_trace.py 20 $O/trace_s0.npy || exit $?
LIFE_MI355X_LIB=build_exp/tr3/liblife_mi355x.so LIFE_SKEW=1 $S 120 $O/trace_s1.log python -u scripts/wg_trace.py 20 $O/trace_s1.npy || exit $?
for i in 1 2; do
  LIFE_SKEW=0 $S 150 $O/base_$i.log $B || exit $?
  LIFE_MI355X_LIB=build_exp/f3/liblife_mi355x.so LIFE_SKEW=1 $S 150 $O/f3_$i.log $B || exit $?
done
echo done
