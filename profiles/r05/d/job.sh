#!/bin/bash
# r05d: the gaps in the partitioned schedule (r05c trace: ~10 us between the
# deep-halo passes, ~30 us from the halo's end to the next pass).
# Expectation: the per-launch timing events (hipExtLaunchKernel start/stop,
# LIFE_TIMING_MODE 2 path) cause the 10 us gaps -- a single-stream call with
# one event pair per call has none (r04 ae trace); the 30 us gap is the
# cross-queue join (compute stream waiting on the interior / halo events).
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r05/d; mkdir -p $O
S=scripts/gpu_step.sh
B="python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 96 --warmup 32"
for sh in 16384x32768 65536x65536; do
  for t in 0 3 0 3; do
    LIFE_TIMING_MODE=$t $S 150 $O/loop_${sh}_t$t.log $B --shape $sh || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp && cd $R
LIFE_TIMING_MODE=3 $S 150 $O/trace_t3.log timeout -s KILL 140 rocprofv3 --kernel-trace -d $O/trace_t3 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 96 --warmup 32 --shape 16384x32768 || exit $?
echo done
