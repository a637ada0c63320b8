#!/bin/bash
# Temporal byte kernel: parity suite, rows sweep (byte), byte/bit bench lines.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r1l; mkdir -p $O
S=scripts/gpu_step.sh
$S 400 $O/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
tail -3 $O/pytest_gpu.log
$S 240 $O/tune_byte.log python -u scripts/tune.py --kernels byte --temporal 32,48,64,96 --gens 2
cat $O/tune_byte.log
$S 240 $O/bench_byte.log python -u bench.py --kernel byte --no-cpu-baseline
grep '^{' $O/bench_byte.log | cut -c1-300
$S 240 $O/bench_bit.log python -u bench.py --no-cpu-baseline
grep '^{' $O/bench_bit.log | cut -c1-300
