#!/bin/bash
# r04ab: byte tiles with the left-neighbour permutes issued 2 / 4 rows ahead
# of their use (LIFE_BYTE_BP_AHEAD, rows fenced in order), and 4 ahead at 3
# tiles per CU; the byte tile's phases were load 33 / generations 93 /
# stores 4 us (r04aa timeline): the generations are latency-bound.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04/ab; mkdir -p $O
S=scripts/gpu_step.sh
B="python -u bench.py --kernel byte --steps 64 --warmup 32 --no-cpu-baseline"
for v in ah2 ah4 ah4w6; do
  LIFE_MI355X_LIB=build_exp/$v/liblife_mi355x.so $S 300 $O/test_$v.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k byte || exit $?
done
for i in 1 2; do
  $S 200 $O/base_$i.log $B || exit $?
  for v in ah2 ah4 ah4w6; do LIFE_MI355X_LIB=build_exp/$v/liblife_mi355x.so $S 200 $O/${v}_$i.log $B || exit $?; done
done
echo done
