#!/bin/bash
# r05j: the dataflow tiles' generation loop with each row's permutes issued
# one row ahead (LIFE_FLOW_BP_AHEAD=1; the compiler had put every permute
# right before its wait there: mean distance 1.8 instructions against 7.6-9.8
# in the per-launch tiles -- the 8 % scheduling loss of round 4 -- which is
# why a dataflow item's body took 60-71 us against 46-52 us for a per-launch
# tile, r05c).  Expectation: dataflow lines +5-10 %; 32768^2 past 0.43 of
# VALU, 65536^2 flow near the tiles.  A/B against builds with 0 and 2 rows
# ahead; flow parity tests first, the whole suite last.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r05/j; mkdir -p $O
S=scripts/gpu_step.sh
$S 400 $O/test_flow.log python -u -m pytest tests/test_gpu_flow.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/test_flow.log && ! grep -q -E "[0-9]+ (failed|error)" $O/test_flow.log || exit 1
B="python -u bench.py --no-cpu-baseline --flow 1"
for sh in 32768x32768 16384x32768 32768x65536 65536x65536; do
  $S 120 $O/a1_$sh.log $B --shape $sh || exit $?
  LIFE_MI355X_LIB=build_exp/fa0/liblife_mi355x.so $S 120 $O/a0_$sh.log $B --shape $sh || exit $?
  LIFE_MI355X_LIB=build_exp/fa2/liblife_mi355x.so $S 120 $O/a2_$sh.log $B --shape $sh || exit $?
  $S 120 $O/tiles_$sh.log $B --shape $sh --flow 0 || exit $?
done
$S 1100 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
echo done
