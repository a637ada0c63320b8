#!/bin/bash
# r2p: dataflow tiles (LIFE_OPT_FLOW): parity, then A/B vs per-launch tiles at 65536^2 / 32768^2 over pass sizes
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2p
mkdir -p $O
S=scripts/gpu_step.sh
$S 400 $O/pytest_flow.log python -u -m pytest tests/test_gpu_flow.py -m gpu -x -v --timeout 120 --timeout-method thread || exit $?
grep -q " passed" $O/pytest_flow.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest_flow.log || exit 1
B="python -u bench.py --no-cpu-baseline --steps 480 --warmup 48"
for round in 1 2; do
  for size in 65536 32768; do
    $S 120 $O/tiles_${size}_m20_$round.json env LIFE_BLOCK_GENS=20 $B --size $size --flow 0 || exit $?
    for m in 8 10 16 20; do
      $S 120 $O/flow1_${size}_m${m}_$round.json env LIFE_BLOCK_GENS=$m $B --size $size --flow 1 || exit $?
    done
    $S 120 $O/flow2_${size}_m16_$round.json env LIFE_BLOCK_GENS=16 $B --size $size --flow 2 || exit $?
  done
done
$S 120 $O/flow1_driver_m10.json env LIFE_BLOCK_GENS=10 python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --flow 1 || exit $?
