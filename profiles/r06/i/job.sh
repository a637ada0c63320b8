#!/bin/bash
# r06i: pass length of the per-launch tiles at 65536^2 (LIFE_BLOCK_GENS).
# Model (life::tail_plan, the banded half tail, c = 0.06; per generation
# makespan(m) * (c + (1 - c) m / 12) / m in full-tile times): m = 12 is 6647
# items = 8.65 rounds that no split improves (9.00 -> 0.750 per generation),
# m = 10 splits to 8.59 (0.724), m = 9 8.53 (0.725), m = 8 8.53 (0.732).
# Expectation: the 992-generation default line +3 % at m = 10 or 9 against
# 12; the deep-halo loopback (11 + 11 + 10 -> 8 + 8 + 8 + 8 at a cap of 10)
# +1-2 %.  (The driver's 20-generation call already runs 10 + 10.)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06/i; mkdir -p $O
S=scripts/gpu_step.sh
U="python -u bench.py --no-cpu-baseline"
L="python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity"
for i in 1 2; do
  for m in 12 10 9 8; do
    LIFE_BLOCK_GENS=$m $S 150 $O/u992_65536_m${m}_$i.log $U || exit $?
  done
  for m in 12 10; do
    LIFE_BLOCK_GENS=$m $S 150 $O/l992_65536_xy_m${m}_$i.log $L --loopback-axes xy || exit $?
  done
done
for m in 12 10; do
  LIFE_BLOCK_GENS=$m $S 150 $O/u992_16384x32768_m${m}.log $U --shape 16384x32768 || exit $?
done
echo done
