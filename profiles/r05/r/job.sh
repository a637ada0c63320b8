#!/bin/bash
# r05r: the driver's call (65536^2, 20 generations from generation 5) as one
# dataflow launch of 2 x 10 generations against the per-launch tiles (two
# launches of 10).  Round 3 measured the dataflow form 38 % slower for 2-3
# passes (0.58 vs 0.42 ms per pass, profiles/r03/r4d) before its permutes-
# ahead and banded-item fixes (+3.5-8 %, r05j).  Expectation: still 10-30 %
# slower (pass-1 items wait for pass-0 neighbours finishing in the same
# round); this decides whether per-item latency work on the dataflow form
# could ever serve the headline shape.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/r; mkdir -p $O
S=scripts/gpu_step.sh
B="python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
for i in 1 2; do
  $S 120 $O/tiles_$i.log $B || exit $?
  LIFE_FLOW_MIN_PASSES=2 LIFE_BLOCK_GENS=10 $S 120 $O/flow10_$i.log $B --flow 1 || exit $?
done
LIFE_FLOW_MIN_PASSES=2 LIFE_BLOCK_GENS=5 $S 120 $O/flow5.log $B --flow 1 || exit $?
echo done
