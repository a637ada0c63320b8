#!/bin/bash
# r05e: the restructured exchange block (halo behind the ring in the compute
# stream's queue, one cross-queue wait placed on the stream predicted to end
# first, LIFE_JOIN 0 auto / 1 halo side / 2 interior side) and the span-only
# timed call of multi-stream steps.  Expectation: the 7 + 12 + 20 us of gaps
# per 32-generation period at 16384x32768 (r05d) shrink; loopback lines
# rise ~5-10 % at the small shapes, ~2 % at 65536^2.  Then the whole GPU suite.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r05/e; mkdir -p $O
S=scripts/gpu_step.sh
B="python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 96 --warmup 32"
for sh in 16384x32768 32768x32768 32768x65536 65536x65536; do
  for j in 0 1 2; do
    LIFE_JOIN=$j $S 150 $O/loop_${sh}_j$j.log $B --shape $sh || exit $?
  done
done
$S 150 $O/loop20_65536.log python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 20 --warmup 5 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $R
$S 150 $O/trace_loop.log timeout -s KILL 140 rocprofv3 --kernel-trace -d $O/trace_loop -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 96 --warmup 32 --shape 16384x32768 || exit $?
$S 1100 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
echo done
