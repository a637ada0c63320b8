#!/bin/bash
# r05f: where the dataflow items lose time (r05c: an item's body takes 60-71
# us at the median against 46-52 us for a per-launch tile).  Timing-only
# builds (results may be stale): LIFE_FLOW_EXP 1 plain window loads instead of
# sc1, 2 plain stores instead of write-through, 4 no store drain before the
# hand-off, 7 all three.  Expectation: one of them recovers most of the
# 25-40 % -- that is the cost to attack (the product keeps sc1 + drain).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/f; mkdir -p $O
S=scripts/gpu_step.sh
B="python -u bench.py --no-cpu-baseline --flow 1"
for sh in 32768x32768 16384x32768 65536x65536; do
  $S 120 $O/base_$sh.log $B --shape $sh || exit $?
  for v in fx1 fx2 fx4 fx7; do
    LIFE_MI355X_LIB=build_exp/$v/liblife_mi355x.so $S 120 $O/${v}_$sh.log $B --shape $sh || exit $?
  done
done
echo done
