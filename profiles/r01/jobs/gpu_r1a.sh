#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r1a; mkdir -p $O
S=scripts/gpu_step.sh
rocm-smi --showproductname > $O/smi.txt 2>&1 || true
$S 420 $O/pytest_gpu.log python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
$S 240 $O/bench_bit.log python -u bench.py --steps 50 --warmup 5 --kernel bit --cpu-seconds 5
$S 240 $O/bench_byte.log python -u bench.py --steps 20 --warmup 3 --kernel byte --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
$GRAFT_REPO_ROOT/$S 240 $GRAFT_REPO_ROOT/$O/rocprof_bit.log rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_bit -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 2 --kernel bit --no-cpu-baseline
