#!/bin/bash
# r05w: the second compute stream and the comm stream get their first
# dispatch at shard creation.  In the driver-shaped RCCL-loopback line (and
# the 8-GPU driver run) the 5-generation warm-up uses the compute stream
# only, so the timed call's exchange block was the interior stream's first
# dispatch.  Expectation: if binding a hardware queue costs ~100 us, the
# 20-generation loopback line gains ~10 % (94.8 T in r05l); otherwise flat.
# The 96-generation loopback lines (their warm-up already overlaps) should
# not move.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/w; mkdir -p $O
S=scripts/gpu_step.sh
$S 400 $O/test_loop.log python -u -m pytest tests/test_gpu_loopback.py tests/test_gpu_parity.py -k "loopback or multi_shard or deep_halo_exchange" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/test_loop.log && ! grep -q -E "[0-9]+ (failed|error)" $O/test_loop.log || exit 1
for i in 1 2 3; do
  $S 150 $O/loop20_$i.log python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 20 --warmup 5 || exit $?
done
$S 300 $O/weak8.log python -u bench.py --gpus 8 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
$S 150 $O/loop_16384x32768.log python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 96 --warmup 32 --shape 16384x32768 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
$S 150 $O/trace_loop20.log timeout -s KILL 140 rocprofv3 --kernel-trace -d $O/trace_loop20 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 20 --warmup 5 || exit $?
echo done
