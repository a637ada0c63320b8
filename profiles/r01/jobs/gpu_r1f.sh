#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r1f; mkdir -p $O
S=scripts/gpu_step.sh
$S 600 $O/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tail -15 $O/pytest_gpu.log
$S 300 $O/tune_t.log python -u scripts/tune.py --temporal 48,64,80,96 --gens 4
cat $O/tune_t.log
$S 240 $O/bench_bit.log python -u bench.py --kernel bit --no-cpu-baseline
grep '^{' $O/bench_bit.log | cut -c1-300
