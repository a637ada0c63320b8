#!/bin/bash
# Byte temporal at K=32 vs 16: parity suite, rows sweep, bench lines.
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r1m; mkdir -p $O
S=scripts/gpu_step.sh
$S 400 $O/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
tail -3 $O/pytest_gpu.log
$S 240 $O/tune_byte_k32.log python -u scripts/tune.py --kernels byte --temporal 32,48,64,80 --gens 2
cat $O/tune_byte_k32.log
LIFE_TEMPORAL_DEPTH_BYTE=16 $S 240 $O/tune_byte_k16.log python -u scripts/tune.py --kernels byte --temporal 32,64 --gens 2
cat $O/tune_byte_k16.log
LIFE_TEMPORAL_DEPTH=32 $S 240 $O/tune_bit_k32.log python -u scripts/tune.py --kernels bit --temporal 64,80,96 --gens 2
cat $O/tune_bit_k32.log
$S 240 $O/bench_byte.log python -u bench.py --kernel byte --no-cpu-baseline
grep '^{' $O/bench_byte.log | cut -c1-300
