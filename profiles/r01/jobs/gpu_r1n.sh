#!/bin/bash
# K=32 defaults (bit 96 rows, byte 48 rows): parity suite, finer rows sweeps, bench lines.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r1n; mkdir -p $O
S=scripts/gpu_step.sh
$S 400 $O/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
tail -3 $O/pytest_gpu.log
$S 240 $O/tune_bit_k32.log python -u scripts/tune.py --kernels bit --temporal 32,48,64,80,96 --gens 2 --rounds 3
cat $O/tune_bit_k32.log
$S 240 $O/tune_byte_k32.log python -u scripts/tune.py --kernels byte --temporal 32,48,64,80,96 --gens 2 --rounds 3
cat $O/tune_byte_k32.log
$S 240 $O/bench_bit.log python -u bench.py
grep '^{' $O/bench_bit.log | cut -c1-300
$S 240 $O/bench_byte.log python -u bench.py --kernel byte --no-cpu-baseline
grep '^{' $O/bench_byte.log | cut -c1-300
