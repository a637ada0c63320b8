#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r1e; mkdir -p $O
S=scripts/gpu_step.sh
$S 600 $O/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tail -15 $O/pytest_gpu.log
$S 120 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
tail -2 $O/smoke.log
$S 240 $O/bench_bit.log python -u bench.py --kernel bit --no-cpu-baseline
grep '^{' $O/bench_bit.log | cut -c1-400
