#!/bin/bash
# r06a: first round-6 job.
# (0) The new parity tests first (persistent interior, one-axis loopback,
#     one-generation fence, timing-off booking): stop before any bench if red.
# (1) VERDICT r5 item 5, headline drift: the round-4 library (31896c8, built
#     from its own tree into build_exp/r4) against HEAD at the driver shape,
#     ABAB twice, same box.  Expectation: equal within ~1 %.
# (2) VERDICT r5 items 1 + 3: every per-GPU block as an RCCL-loopback line
#     (only the axes its N partitions: x for N = 2's {2,1}) beside the
#     unpartitioned line of the SAME shape and --steps / --warmup, and the
#     loopback once more with the one-shot interior (LIFE_PERSIST_RESERVE=0,
#     the round-5 schedule).  Expectation: the persistent interior (default,
#     8 slots left free) shortens the 65536^2 exchange block (RCCL kernel
#     ~15 us instead of ~300 beside the interior), 65536^2 xy loopback /
#     unpartitioned from ~0.90-0.95 towards ~0.97; 16384x32768 unchanged
#     (584 interior tiles < 760: one-shot either way).
# (3) Kernel traces of the 96-generation 65536^2 loopback, persistent and
#     one-shot (the ~0.7 ms r05's phases did not account for).
# (4) The whole GPU suite.  Expectation: green.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r06/a; mkdir -p $O
S=scripts/gpu_step.sh
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider"
$S 120 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
$S 400 $O/pytest_new.log $T tests/test_gpu_loopback.py tests/test_gpu_parity.py -m gpu -k "persistent or one_axis or onegen_wide or timing_mode_off" || exit $?
grep -q " passed" $O/pytest_new.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest_new.log || exit 1
D="python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
for i in 1 2; do
  LIFE_MI355X_LIB=$R/build_exp/r4/liblife_mi355x.so $S 120 $O/drv_r4_$i.log $D || exit $?
  $S 120 $O/drv_head_$i.log $D || exit $?
done
U="python -u bench.py --no-cpu-baseline"
L="python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity"
for i in 1 2; do
  $S 120 $O/u20_65536_$i.log $U --steps 20 --warmup 5 || exit $?
  for ax in xy x; do
    $S 120 $O/l20_65536_${ax}_$i.log $L --steps 20 --warmup 5 --loopback-axes $ax || exit $?
    LIFE_PERSIST_RESERVE=0 $S 120 $O/l20_65536_${ax}_oneshot_$i.log $L --steps 20 --warmup 5 --loopback-axes $ax || exit $?
  done
done
for sa in 65536x65536:xy 65536x65536:x 32768x65536:x 32768x32768:xy 16384x32768:xy; do
  sh=${sa%%:*}; ax=${sa##*:}
  for i in 1 2; do
    $S 150 $O/u992_${sh}_${ax}_$i.log $U --shape $sh || exit $?
    $S 150 $O/l992_${sh}_${ax}_$i.log $L --shape $sh --loopback-axes $ax || exit $?
    LIFE_PERSIST_RESERVE=0 $S 150 $O/l992_${sh}_${ax}_oneshot_$i.log $L --shape $sh --loopback-axes $ax || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp && cd $R
$S 150 $O/trace_loop96.log timeout -s KILL 140 rocprofv3 --kernel-trace --stats -d $O/trace_loop96 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 96 --warmup 32 || exit $?
LIFE_PERSIST_RESERVE=0 $S 150 $O/trace_loop96_oneshot.log timeout -s KILL 140 rocprofv3 --kernel-trace --stats -d $O/trace_loop96_oneshot -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 96 --warmup 32 || exit $?
$S 1100 $O/pytest.log $T tests -m gpu || exit $?
grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
echo done
