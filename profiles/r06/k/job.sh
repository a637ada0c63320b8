#!/bin/bash
# r06k: 26-row bit tiles (8 waves x 26 pair rows = 208-row window, 79 VGPRs,
# no scratch, still 3 workgroups per CU) against the shipped 24-row tiles
# (LIFE_TEMPORAL_ROWS 26 / 24).  Model (life::tail_plan): 16384x32768 at
# m = 12 is 761 items = ONE round (1.08 tile-times of a 24-row tile against
# 1.53); 32768^2 tiles 2 rounds (2.17 against 2.53); 65536^2 m = 12 7.9
# rounds (8.67 against 9.00), m = 10 ~8.45 against 8.59.  Expectation:
# 16384x32768 +25-40 %, 32768^2 tiles +10-15 %, 65536^2 992 gens +3 %,
# driver line +1-2 %; the dataflow instance spills at 26 rows (24-60 B
# scratch): flow lines slower.  Parity subset under 26 after the lines.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/k; mkdir -p $O
S=scripts/gpu_step.sh
T="python -u -m pytest -x -q --timeout 600 --timeout-method thread -p no:cacheprovider"
U="python -u bench.py --no-cpu-baseline"
L="python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity"
for i in 1 2; do
  for r in 24 26; do
    LIFE_TEMPORAL_ROWS=$r $S 120 $O/drv_r${r}_$i.log $U --steps 20 --warmup 5 || exit $?
    LIFE_TEMPORAL_ROWS=$r $S 150 $O/u992_65536_r${r}_$i.log $U || exit $?
    LIFE_TEMPORAL_ROWS=$r $S 150 $O/u992_16384x32768_r${r}_$i.log $U --shape 16384x32768 --flow 0 || exit $?
    LIFE_TEMPORAL_ROWS=$r $S 150 $O/u992_32768_tiles_r${r}_$i.log $U --shape 32768x32768 --flow 0 || exit $?
    LIFE_TEMPORAL_ROWS=$r $S 150 $O/u992_32768x65536_tiles_r${r}_$i.log $U --shape 32768x65536 --flow 0 || exit $?
    LIFE_TEMPORAL_ROWS=$r $S 150 $O/l992_16384x32768_xy_r${r}_$i.log $L --shape 16384x32768 --loopback-axes xy || exit $?
    LIFE_TEMPORAL_ROWS=$r $S 150 $O/l992_65536_x_r${r}_$i.log $L --loopback-axes x || exit $?
  done
done
for r in 24 26; do
  LIFE_TEMPORAL_ROWS=$r $S 150 $O/u992_32768_flow_r${r}.log $U --shape 32768x32768 --flow 1 || exit $?
done
LIFE_TEMPORAL_ROWS=26 $S 600 $O/pytest26.log $T tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_loopback.py -m gpu -k "band or tail or driver_shape or random_shapes or parity or loopback or deep" || exit $?
grep -q " passed" $O/pytest26.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest26.log || exit 1
echo done
