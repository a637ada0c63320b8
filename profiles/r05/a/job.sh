#!/bin/bash
# r05a: the shape landscape.  Single-GPU lines at the
# per-GPU blocks of configs[2]/[3]: 32768^2, 32768x65536, 16384x32768, with
# the per-launch tiles (default), the dataflow form (flow 1/2), generations per
# pass 8-16, tile shapes, the tail split off; RCCL-loopback lines (phases) at
# the three shapes; a per-workgroup timeline at 32768^2.
# Expectation: the tiles lose 25-30 % to the launch tail at 32768^2 (0.383 vs
# 0.446 of VALU at 65536^2) and more at 16384x32768 (~1.08 rounds of 768
# slots per launch); the dataflow form, which has no launch boundary, should
# win there by about that much (it lost 3-5 % at 65536^2).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/a; mkdir -p $O
S=scripts/gpu_step.sh
B="python -u bench.py --no-cpu-baseline"
for sh in 32768x32768 32768x65536 16384x32768; do
  $S 120 $O/tiles_$sh.log $B --shape $sh || exit $?
  $S 120 $O/flow1_$sh.log $B --shape $sh --flow 1 || exit $?
  $S 120 $O/flow2_$sh.log $B --shape $sh --flow 2 || exit $?
  $S 120 $O/tiles20_$sh.log $B --shape $sh --steps 20 --warmup 5 || exit $?
  $S 150 $O/loop_$sh.log $B --shape $sh --rank-mode --loopback --no-parity --steps 96 --warmup 32 || exit $?
done
for m in 8 10 11 14 16; do
  LIFE_BLOCK_GENS=$m $S 120 $O/m${m}_32768.log $B --shape 32768x32768 || exit $?
  LIFE_BLOCK_GENS=$m $S 120 $O/m${m}_16384x32768.log $B --shape 16384x32768 || exit $?
done
LIFE_TAIL_SPLIT=0 $S 120 $O/notail_32768.log $B --shape 32768x32768 || exit $?
for rw in 16x16 24x12 32x8 16x8; do
  R=${rw%x*}; NW=${rw#*x}
  LIFE_TEMPORAL_ROWS=$R LIFE_TILE_WAVES=$NW $S 120 $O/shape${rw}_32768.log $B --shape 32768x32768 || exit $?
done
$S 120 $O/tiles_65536.log $B || exit $?
$S 120 $O/flow1_65536.log $B --flow 1 || exit $?
WG_TRACE_SHAPE=32768x32768 LIFE_MI355X_LIB=build_exp/wgt/liblife_mi355x.so $S 120 $O/wgtrace_32768.log python -u scripts/wg_trace.py 12 || exit $?
echo done
