#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r1b; mkdir -p $O
S=scripts/gpu_step.sh
$S 420 $O/pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
tail -3 $O/pytest_gpu.log
$S 300 $O/tune.log python -u scripts/tune.py
cat $O/tune.log
for m in lib_only lib_then_torch torch_then_lib torch_cuda; do $S 120 $O/probe_$m.log python -u scripts/torch_probe.py $m; tail -2 $O/probe_$m.log; done
$S 240 $O/bench_bit.log python -u bench.py --steps 100 --warmup 5 --kernel bit --cpu-seconds 5
tail -2 $O/bench_bit.log
