#!/bin/bash
# r04v: byte tiles at 3 per CU -- LIFE_BYTE_WPE=6 fits R = 48 in 74 VGPRs
# without spills once the window load is fenced every 4 (or 2) rows
# (LIFE_BYTE_LOAD_CHUNK); against the shipped 2 per CU, and the chunked load
# alone.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04/v; mkdir -p $O
S=scripts/gpu_step.sh
B="python -u bench.py --kernel byte --steps 64 --warmup 32 --no-cpu-baseline"
for v in w6c4 w6c2; do
  LIFE_MI355X_LIB=build_exp/$v/liblife_mi355x.so $S 300 $O/test_$v.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k byte || exit $?
done
for i in 1 2; do
  $S 200 $O/base_$i.log $B || exit $?
  for v in w4c4 w6c4 w6c2; do LIFE_MI355X_LIB=build_exp/$v/liblife_mi355x.so $S 200 $O/${v}_$i.log $B || exit $?; done
done
echo done
