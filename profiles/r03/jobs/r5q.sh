#!/bin/bash
# r5q: generations per launch (LIFE_BLOCK_GENS) for the 992-generation default run with the XCD order.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5q
mkdir -p $O
S=scripts/gpu_step.sh
for i in 1 2; do
  for m in 8 10 12 14; do
    LIFE_BLOCK_GENS=$m $S 200 $O/def_m${m}_$i.json python -u bench.py --no-cpu-baseline || exit $?
  done
done
echo done
