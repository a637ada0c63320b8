#!/bin/bash
# r2q: dataflow tiles, pass size m and tile height R sweep at 65536^2 / 32768^2 (two interleaved rounds)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2q
mkdir -p $O
S=scripts/gpu_step.sh
B="python -u bench.py --no-cpu-baseline --steps 480 --warmup 48 --flow 1"
for round in 1 2; do
  for size in 65536 32768; do
    for m in 20 24 28 32; do
      $S 120 $O/R48_${size}_m${m}_$round.json env LIFE_BLOCK_GENS=$m $B --size $size || exit $?
    done
    for m in 20 24; do
      $S 120 $O/R40_${size}_m${m}_$round.json env LIFE_TEMPORAL_ROWS=40 LIFE_BLOCK_GENS=$m $B --size $size || exit $?
    done
  done
done
$S 300 $O/default_flow.json python -u bench.py --no-cpu-baseline --flow 1 || exit $?
$S 300 $O/default_flow_32768.json python -u bench.py --no-cpu-baseline --flow 1 --size 32768 || exit $?
