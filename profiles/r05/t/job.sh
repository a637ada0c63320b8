#!/bin/bash
# r05t: generations per pass for the dataflow form at configs[2] (32768^2).
# A dataflow item pays a flag poll, a window load and a flagged store per
# pass; more generations per pass amortise them against more ghost rows
# (per-launch tiles were flat over m = 8-16, r05a; the dataflow form was
# only run at m = 12).  Expectation: m = 14-16 +1-3 % if the per-item fixed
# cost is what keeps the dataflow items ~20 % longer than per-launch tiles.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/t; mkdir -p $O
S=scripts/gpu_step.sh
for i in 1 2; do
  for m in 12 14 16 10; do
    LIFE_BLOCK_GENS=$m $S 120 $O/c2_m${m}_$i.log python -u bench.py --no-cpu-baseline --shape 32768x32768 --flow 1 || exit $?
  done
done
for m in 12 14 16; do
  LIFE_BLOCK_GENS=$m $S 120 $O/c3n2_m$m.log python -u bench.py --no-cpu-baseline --shape 32768x65536 --flow 1 || exit $?
done
echo done
