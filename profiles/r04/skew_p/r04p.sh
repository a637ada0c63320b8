#!/bin/bash
# r04p: skewed tiles with the generation barrier pinned after the publish
# (LIFE_SKEW_FENCE=1) and with the rows above read right after it (=2),
# against the in-tree build (the compiler sinks the barrier).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04/p; mkdir -p $O
S=scripts/gpu_step.sh
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline"
for v in f1 f2; do
  LIFE_MI355X_LIB=build_exp/$v/liblife_mi355x.so LIFE_SKEW=1 $S 120 $O/test_$v.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k skew || exit $?
done
for i in 1 2; do
  LIFE_SKEW=0 $S 150 $O/base_$i.log $B || exit $?
  LIFE_SKEW=1 $S 150 $O/f0_$i.log $B || exit $?
  for v in f1 f2; do LIFE_MI355X_LIB=build_exp/$v/liblife_mi355x.so LIFE_SKEW=1 $S 150 $O/${v}_$i.log $B || exit $?; done
done
echo done
