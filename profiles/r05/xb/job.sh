#!/bin/bash
# r05xb: is the halo beside the interior starved of dispatch?  r05w's trace:
# the RCCL kernel started right after the pack but ended 308 us later, within
# 4 us of the interior's end (14 us when it runs alone) -- as if some of its
# workgroups could not be dispatched until the interior's last tiles were.
# The current schedule with LIFE_STREAM_PRIORITY=1 (ring + halo stream at the
# greatest HIP priority, interior at the least; round 4 measured it under the
# old three-stream schedule).  Expectation: if queue priority orders the
# dispatch, the halo beside a 65536^2 interior drops from ~0.3-0.4 ms towards
# its ~0.05 ms alone and 16384x32768's block shrinks; else no change.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/xb; mkdir -p $O
S=scripts/gpu_step.sh
for p in 0 1; do
  LIFE_STREAM_PRIORITY=$p $S 150 $O/loop20_p$p.log python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 20 --warmup 5 || exit $?
  LIFE_STREAM_PRIORITY=$p $S 150 $O/loop_16384x32768_p$p.log python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 96 --warmup 32 --shape 16384x32768 || exit $?
  LIFE_STREAM_PRIORITY=$p $S 150 $O/loop_65536_p$p.log python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 96 --warmup 32 || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
LIFE_STREAM_PRIORITY=1 $S 150 $O/trace_p1.log timeout -s KILL 140 rocprofv3 --kernel-trace -d $O/trace_p1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 20 --warmup 5 || exit $?
echo done
