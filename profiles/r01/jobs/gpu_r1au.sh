#!/bin/bash
# Final round-1 check at HEAD: full GPU suite, smoke, bench bit/byte at the defaults.
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1au; mkdir -p $O
S=$R/scripts/gpu_step.sh
$S 900 $O/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread
tail -3 $O/pytest_gpu.log
grep -q " passed" $O/pytest_gpu.log && ! grep -q "failed" $O/pytest_gpu.log
$S 200 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
$S 200 $O/bench_bit.log python -u bench.py
$S 200 $O/bench_byte.log python -u bench.py --kernel byte --no-cpu-baseline
cat $O/bench_bit.log $O/bench_byte.log
export TMPDIR=/tmp
