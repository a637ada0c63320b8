#!/bin/bash
# Stacked-wave temporal kernel: parity suite, then rows-per-wave x K sweep, bench.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r1j; mkdir -p $O
S=scripts/gpu_step.sh
$S 300 $O/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
tail -3 $O/pytest_gpu.log
$S 240 $O/tune_k8.log python -u scripts/tune.py --temporal 32,48,64,80,96 --gens 4
cat $O/tune_k8.log
LIFE_TEMPORAL_DEPTH=16 $S 240 $O/tune_k16.log python -u scripts/tune.py --temporal 32,48,64,80,96 --gens 2
cat $O/tune_k16.log
$S 240 $O/bench_bit.log python -u bench.py --no-cpu-baseline
grep '^{' $O/bench_bit.log | cut -c1-400
