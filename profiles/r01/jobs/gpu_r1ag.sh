#!/bin/bash
# Re-validation at HEAD after a container rebuild: full GPU suite, smoke, default bench, rocprof stats.
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1ag; mkdir -p $O
S=$R/scripts/gpu_step.sh
$S 900 $O/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread
tail -3 $O/pytest_gpu.log
$S 200 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
tail -2 $O/smoke.log
$S 300 $O/bench.log python -u bench.py
cat $O/bench.log
export TMPDIR=/tmp
$S 300 $O/rocprof.log rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --no-cpu-baseline
tail -3 $O/rocprof.log
