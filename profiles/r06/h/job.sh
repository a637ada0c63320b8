#!/bin/bash
# r06h: the flags of the events that order a shard's ring / halo stream and
# its interior stream (LIFE_SYNC_EVENTS 0 = HIP default, system-scope fence;
# 1 = hipEventDisableSystemFence; 2 = hipEventReleaseToDevice).  The r06d
# 16384x32768 loopback trace has 7-9 us between the last plain pass and the
# ring of each exchange block (the ev_entry record between them) and ~10 us
# from the block's end to the next pass, where back-to-back passes have none:
# ~17 us per 32 generations (~250 us), ~7 %.  Expectation: if the system-scope
# fence is the gap, flag 1 or 2 gives the 16384x32768 loopback +3-7 %,
# 32768^2 +2-4 %, 65536^2 ~+1 %; parity green with both flags.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r06/h; mkdir -p $O
S=scripts/gpu_step.sh
T="python -u -m pytest -x -q --timeout 600 --timeout-method thread -p no:cacheprovider"
for f in 1 2; do
  LIFE_SYNC_EVENTS=$f $S 400 $O/pytest_ev$f.log $T tests/test_gpu_loopback.py tests/test_gpu_parity.py -m gpu -k "loopback or overlap or deep or onegen or exchange or rank" || exit $?
  grep -q " passed" $O/pytest_ev$f.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest_ev$f.log || exit 1
done
L="python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity"
for i in 1 2; do
  for f in 0 1 2; do
    LIFE_SYNC_EVENTS=$f $S 150 $O/l992_16384x32768_xy_ev${f}_$i.log $L --shape 16384x32768 --loopback-axes xy || exit $?
    LIFE_SYNC_EVENTS=$f $S 150 $O/l992_32768x32768_xy_ev${f}_$i.log $L --shape 32768x32768 --loopback-axes xy || exit $?
    LIFE_SYNC_EVENTS=$f $S 150 $O/l992_65536_x_ev${f}_$i.log $L --loopback-axes x || exit $?
    LIFE_SYNC_EVENTS=$f $S 120 $O/l20_65536_xy_ev${f}_$i.log $L --steps 20 --warmup 5 --loopback-axes xy || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp && cd $R
for f in 0 1; do
  LIFE_SYNC_EVENTS=$f $S 150 $O/trace_ev$f.log timeout -s KILL 140 rocprofv3 --kernel-trace --stats -d $O/trace_ev$f -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --shape 16384x32768 --steps 96 --warmup 32 || exit $?
done
echo done
