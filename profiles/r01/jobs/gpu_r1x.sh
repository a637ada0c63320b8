#!/bin/bash
# Restored-tree check: full GPU suite (incl. rank mode / torchrun bootstrap),
# smoke, default bench line.
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1x; mkdir -p $O
S=$R/scripts/gpu_step.sh
$S 200 $O/pytest_rank.log python -u -m pytest tests/test_gpu_rank.py -m gpu -v --timeout 240 --timeout-method thread
tail -8 $O/pytest_rank.log
$S 500 $O/pytest_gpu.log python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread
tail -4 $O/pytest_gpu.log
$S 120 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
tail -1 $O/smoke.log
$S 240 $O/bench_bit.log python -u bench.py
grep '^{' $O/bench_bit.log
