#!/bin/bash
# configs[2]: random 50% 32768^2, generations 32..1024, bit vs byte.
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1aw; mkdir -p $O
S=$R/scripts/gpu_step.sh
for k in bit byte; do
  $S 200 $O/bench_$k.log python -u bench.py --size 32768 --kernel $k --no-cpu-baseline
  cat $O/bench_$k.log
done
