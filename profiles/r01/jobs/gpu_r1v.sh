#!/bin/bash
# Parity suite + smoke after temporal tiles for widths not a multiple of 32.
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1v; mkdir -p $O
S=$R/scripts/gpu_step.sh
$S 500 $O/pytest_gpu.log python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread
tail -15 $O/pytest_gpu.log
$S 120 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
tail -1 $O/smoke.log
$S 240 $O/bench_bit.log python -u bench.py --no-cpu-baseline
grep '^{' $O/bench_bit.log | cut -c1-300
