#!/bin/bash
# r04z: skewed segments with progress-balanced issue priority
# (LIFE_SKEW_BALANCE=1, build_exp/bal) against the falling-priority form
# (in-tree) and the per-launch tiles; timeline of the balanced form.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04/z; mkdir -p $O
S=scripts/gpu_step.sh
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline"
LIFE_MI355X_LIB=build_exp/bal/liblife_mi355x.so LIFE_SKEW=1 $S 120 $O/test_bal.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "skew or timing_stats" || exit $?
LIFE_MI355X_LIB=build_exp/tbal/liblife_mi355x.so LIFE_SKEW=1 $S 120 $O/trace_bal.log python -u scripts/wg_trace.py 20 $O/trace_bal.npy || exit $?
for i in 1 2; do
  LIFE_SKEW=0 $S 150 $O/base_$i.log $B || exit $?
  LIFE_SKEW=1 $S 150 $O/skew_$i.log $B || exit $?
  LIFE_MI355X_LIB=build_exp/bal/liblife_mi355x.so LIFE_SKEW=1 $S 150 $O/bal_$i.log $B || exit $?
done
echo done
