#!/bin/bash
# r06f: the exchange pass's interior with the banded half-height tail,
# planned with the ring's tiles counted as holding their slots
# (LIFE_INTERIOR_TAIL 1, new) against no split for it (0, rounds 5 / r06d).
# Model: the exchange pass 2.0 -> 1.53 tile-times at 16384x32768, 3.0 ->
# 2.53 at 32768^2.  Expectation: RCCL-loopback lines 16384x32768 +5-8 %,
# 32768^2 +3-6 %, 65536^2 +0-2 %; parity green.  The unpartitioned lines of
# the same shapes and steps alternate with them, so the scaling tables can be
# rebuilt from this job if it is kept (scripts/scaling_table.py).  (The
# whole GPU suite and the trace run in the next job: one call stays under
# 20 minutes.)
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r06/f; mkdir -p $O
S=scripts/gpu_step.sh
T="python -u -m pytest -x -q --timeout 600 --timeout-method thread -p no:cacheprovider"
$S 120 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
$S 600 $O/pytest_new.log $T tests/test_gpu_loopback.py tests/test_gpu_fullsize.py tests/test_gpu_bench.py -m gpu -k "exchange_pass or loopback or c4 or tail or multi_shard_bench or weak_scaling" || exit $?
grep -q " passed" $O/pytest_new.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest_new.log || exit 1
U="python -u bench.py --no-cpu-baseline"
L="python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity"
for i in 1 2; do
  $S 120 $O/u20_65536_$i.log $U --steps 20 --warmup 5 || exit $?
  for t in 1 0; do
    LIFE_INTERIOR_TAIL=$t $S 120 $O/l20_65536_x_it${t}_$i.log $L --steps 20 --warmup 5 --loopback-axes x || exit $?
    LIFE_INTERIOR_TAIL=$t $S 120 $O/l20_65536_xy_it${t}_$i.log $L --steps 20 --warmup 5 --loopback-axes xy || exit $?
  done
  $S 150 $O/u992_65536_$i.log $U || exit $?
  $S 150 $O/u992_32768x65536_$i.log $U --shape 32768x65536 || exit $?
  $S 150 $O/u992_32768x32768_$i.log $U --shape 32768x32768 || exit $?
  $S 150 $O/u992_16384x32768_$i.log $U --shape 16384x32768 || exit $?
  for t in 1 0; do
    LIFE_INTERIOR_TAIL=$t $S 150 $O/l992_65536_x_it${t}_$i.log $L --loopback-axes x || exit $?
    LIFE_INTERIOR_TAIL=$t $S 150 $O/l992_65536_xy_it${t}_$i.log $L --loopback-axes xy || exit $?
    LIFE_INTERIOR_TAIL=$t $S 150 $O/l992_32768x65536_x_it${t}_$i.log $L --shape 32768x65536 --loopback-axes x || exit $?
    LIFE_INTERIOR_TAIL=$t $S 150 $O/l992_32768x32768_xy_it${t}_$i.log $L --shape 32768x32768 --loopback-axes xy || exit $?
    LIFE_INTERIOR_TAIL=$t $S 150 $O/l992_16384x32768_xy_it${t}_$i.log $L --shape 16384x32768 --loopback-axes xy || exit $?
  done
done
echo done
