#!/bin/bash
# r06c: banded partial-height tail tiles.
# LIFE_TAIL_SPLIT 3 (new default): the bottom tile rows of a full-width
# launch as 3/4- and half-height tiles, banded in the last tile column, the
# split chosen by life::tail_plan's list-schedule model; 2 = round 5 (half
# tiles only; now banded too).  Model (c = 0.06): 16384x32768 1.53 -> 1.295
# tile-times per pass (-15 %), 32768^2 / 32768x65536 2.53 -> 2.295 / 4.53 ->
# 4.295 (-9 / -5 %), 65536^2 at m = 12 9.0 -> 8.765 (-2.6 %), at m = 10 (the
# driver's call) unchanged.
# Expectation: 16384x32768 per-launch tiles 0.31-0.32 -> >= 0.36 of VALU;
# loopback lines of the small blocks +5-15 %; default 65536^2 line +1-2 %;
# driver line unchanged; parity green.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r06/c; mkdir -p $O
S=scripts/gpu_step.sh
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
$S 120 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
$S 500 $O/pytest_tail.log $T tests/test_gpu_fullsize.py tests/test_gpu_bench.py -m gpu -k "partial_height or tail_split or driver_shape or single_gpu_line" || exit $?
grep -q " passed" $O/pytest_tail.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest_tail.log || exit 1
U="python -u bench.py --no-cpu-baseline"
L="python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity"
for i in 1 2; do
  for mode in 2 3; do
    LIFE_TAIL_SPLIT=$mode $S 120 $O/drv_t${mode}_$i.log $U --steps 20 --warmup 5 || exit $?
    LIFE_TAIL_SPLIT=$mode $S 150 $O/def_t${mode}_$i.log $U || exit $?
    LIFE_TAIL_SPLIT=$mode $S 150 $O/u16384x32768_t${mode}_$i.log $U --shape 16384x32768 --flow 0 || exit $?
    LIFE_TAIL_SPLIT=$mode $S 150 $O/u32768x32768_t${mode}_$i.log $U --shape 32768x32768 --flow 0 || exit $?
    LIFE_TAIL_SPLIT=$mode $S 150 $O/l16384x32768_t${mode}_$i.log $L --shape 16384x32768 || exit $?
    LIFE_TAIL_SPLIT=$mode $S 150 $O/l32768x32768_t${mode}_$i.log $L --shape 32768x32768 || exit $?
    LIFE_TAIL_SPLIT=$mode $S 150 $O/l32768x65536_x_t${mode}_$i.log $L --shape 32768x65536 --loopback-axes x || exit $?
    LIFE_TAIL_SPLIT=$mode $S 150 $O/l65536_t${mode}_$i.log $L || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp && cd $R
for mode in 2 3; do
  LIFE_TAIL_SPLIT=$mode $S 150 $O/trace_16384_t$mode.log timeout -s KILL 140 rocprofv3 --kernel-trace --stats -d $O/trace_16384_t$mode -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --shape 16384x32768 --flow 0 --steps 96 --warmup 32 || exit $?
done
$S 1100 $O/pytest.log $T tests -m gpu || exit $?
grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
echo done
