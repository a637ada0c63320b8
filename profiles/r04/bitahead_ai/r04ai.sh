#!/bin/bash
# r04ai: bit tiles with the neighbour permutes issued 1 / 2 rows ahead, rows
# fenced in order (LIFE_BIT_BP_AHEAD), against the in-tree build.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04/ai; mkdir -p $O
S=scripts/gpu_step.sh
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline"
for v in bah1 bah2; do
  LIFE_MI355X_LIB=build_exp/$v/liblife_mi355x.so $S 300 $O/test_$v.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "bit and not skew" || exit $?
done
for i in 1 2 3; do
  $S 150 $O/base_$i.log $B || exit $?
  for v in bah1 bah2; do LIFE_MI355X_LIB=build_exp/$v/liblife_mi355x.so $S 150 $O/${v}_$i.log $B || exit $?; done
done
echo done
