#!/bin/bash
# r04ad: per-tile index set-up without 64-bit remainders (LIFE_FAST_WRAP=1:
# one conditional add / subtract for the wrapped pair column and row) --
# parity of the bit and byte paths, then the driver-shaped bit call and the
# byte call against the in-tree build, alternating.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04/ad; mkdir -p $O
S=scripts/gpu_step.sh
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline"
BB="python -u bench.py --kernel byte --steps 64 --warmup 32 --no-cpu-baseline"
L=build_exp/fw/liblife_mi355x.so
LIFE_MI355X_LIB=$L $S 400 $O/test_fw.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_golden.py || exit $?
for i in 1 2 3; do
  $S 150 $O/base_$i.log $B || exit $?
  LIFE_MI355X_LIB=$L $S 150 $O/fw_$i.log $B || exit $?
done
for i in 1 2; do
  $S 200 $O/bbase_$i.log $BB || exit $?
  LIFE_MI355X_LIB=$L $S 200 $O/bfw_$i.log $BB || exit $?
done
echo done
