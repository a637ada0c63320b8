#!/bin/bash
# r05s: 16-row bit tiles at 4 per CU (32 waves per CU, <= 64 VGPRs: the
# R = 16 instance uses 60) against the shipped 24-row tiles at 3 per CU.  The
# 24-row tile issues VALU ~61 % of the held clock; more resident waves may
# hide more of the LDS / barrier latency, against 18.5 % ghost rows instead of
# 10.4 % at m = 10.  Expectation: within -5..+5 %; keep only a same-box gain.
# Then 16 waves x 16 rows at 2 per CU (7.8 % ghost rows, a 16-wave barrier).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/s; mkdir -p $O
S=scripts/gpu_step.sh
$S 300 $O/test_r16.log env LIFE_TEMPORAL_ROWS=16 python -u -m pytest tests/test_gpu_parity.py -k "temporal_single_shard or deep_halo" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/test_r16.log && ! grep -q -E "[0-9]+ (failed|error)" $O/test_r16.log || exit 1
B="python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
for i in 1 2; do
  $S 120 $O/drv_r24_$i.log $B || exit $?
  LIFE_TEMPORAL_ROWS=16 $S 120 $O/drv_r16_$i.log $B || exit $?
done
$S 120 $O/def_r24.log python -u bench.py --no-cpu-baseline || exit $?
LIFE_TEMPORAL_ROWS=16 $S 120 $O/def_r16.log python -u bench.py --no-cpu-baseline || exit $?
for bg in 8 12 16; do
  LIFE_TEMPORAL_ROWS=16 LIFE_BLOCK_GENS=$bg $S 120 $O/def_r16_m$bg.log python -u bench.py --no-cpu-baseline --flow 0 || exit $?
done
$S 120 $O/c2_r24.log python -u bench.py --no-cpu-baseline --shape 32768x32768 --flow 0 || exit $?
LIFE_TEMPORAL_ROWS=16 $S 120 $O/c2_r16.log python -u bench.py --no-cpu-baseline --shape 32768x32768 --flow 0 || exit $?
# 16 waves x 16 rows (256-row windows, 2 per CU, 32 waves): an experimental
# build with that instance (build_exp/w16), same parity subset first
W="env LIFE_MI355X_LIB=build_exp/w16/liblife_mi355x.so LIFE_TILE_WAVES=16 LIFE_TEMPORAL_ROWS=16"
$S 300 $O/test_w16.log $W python -u -m pytest tests/test_gpu_parity.py -k "temporal_single_shard" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/test_w16.log && ! grep -q -E "[0-9]+ (failed|error)" $O/test_w16.log || exit 1
for i in 1 2; do
  $S 120 $O/drv_w16_$i.log $W $B || exit $?
done
$S 120 $O/def_w16.log $W python -u bench.py --no-cpu-baseline || exit $?
$S 120 $O/c2_w16.log $W python -u bench.py --no-cpu-baseline --shape 32768x32768 --flow 0 || exit $?
echo done
