#!/bin/bash
# r6g: r6f's RCCL loopback line read 51.7 T (r6d: 91.5-92.6 T with the same code): repeat it, with and
# without the phase events in the timed call.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6g
rm -rf $O; mkdir -p $O
S=scripts/gpu_step.sh
for i in 1 2 3; do
  for t in 0 1; do
    LIFE_BENCH_PHASES_TIMED=$t $S 200 $O/rccl20_t${t}_$i.json python -u bench.py --rank-mode --loopback --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  done
done
echo done
