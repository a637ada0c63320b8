#!/bin/bash
# r6h: partitioned 20-generation calls (RCCL loopback) as one block of 20 (one halo exchange) against
# two blocks of 10 (two exchanges): data for choosing the block size per schedule.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6h
rm -rf $O; mkdir -p $O
S=scripts/gpu_step.sh
for i in 1 2; do
  for m in 0 20; do
    LIFE_BLOCK_GENS=$m $S 200 $O/rccl20_m${m}_$i.json python -u bench.py --rank-mode --loopback --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  done
done
echo done
