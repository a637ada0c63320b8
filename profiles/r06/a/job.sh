#!/bin/bash
# r06a: first round-6 job.
# (1) VERDICT r5 item 5, headline drift: the round-4 library (31896c8, built
#     from its own tree into build_exp/r4) against HEAD at the driver shape,
#     ABAB twice, same box.  Expectation: equal within ~1 % (the r05 lines sat
#     inside round 4's 96-103.5 T spread).
# (2) VERDICT r5 item 3, controlled scaling predictions: every per-GPU block
#     as an RCCL-loopback line (only the axes its N partitions: x for N = 2's
#     {2,1}) beside the unpartitioned line of the SAME shape and --steps /
#     --warmup, ABAB; 65536^2 (configs[4]'s weak block) at the driver's
#     20-generation shape and at 992 generations.  Expectation: 65536^2 xy
#     loopback / unpartitioned ~0.90-0.95.
# (3) A kernel trace of the 96-generation 65536^2 loopback (the ~0.7 ms the
#     recorded phases did not account for in r05).
# (4) The whole GPU suite with the round-6 tests (one-generation fence,
#     timing-off booking, one-axis loopback).  Expectation: green.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r06/a; mkdir -p $O
S=scripts/gpu_step.sh
$S 120 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
D="python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
for i in 1 2; do
  LIFE_MI355X_LIB=$R/build_exp/r4/liblife_mi355x.so $S 120 $O/drv_r4_$i.log $D || exit $?
  $S 120 $O/drv_head_$i.log $D || exit $?
done
U="python -u bench.py --no-cpu-baseline"
L="python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity"
for i in 1 2; do
  $S 120 $O/u20_65536_$i.log $U --steps 20 --warmup 5 || exit $?
  $S 120 $O/l20_65536_xy_$i.log $L --steps 20 --warmup 5 --loopback-axes xy || exit $?
  $S 120 $O/l20_65536_x_$i.log $L --steps 20 --warmup 5 --loopback-axes x || exit $?
done
for sa in 65536x65536:xy 65536x65536:x 32768x65536:x 32768x32768:xy 16384x32768:xy; do
  sh=${sa%%:*}; ax=${sa##*:}
  for i in 1 2; do
    $S 150 $O/u992_${sh}_${ax}_$i.log $U --shape $sh || exit $?
    $S 150 $O/l992_${sh}_${ax}_$i.log $L --shape $sh --loopback-axes $ax || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp && cd $R
$S 150 $O/trace_loop96.log timeout -s KILL 140 rocprofv3 --kernel-trace --stats -d $O/trace_loop96 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 96 --warmup 32 || exit $?
$S 1100 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
echo done
