#!/bin/bash
# Drifting frame for the byte encoding only: full GPU suite, smoke, bench bit/byte/p46, rocprof stats of bit and byte.
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1aq; mkdir -p $O
S=$R/scripts/gpu_step.sh
$S 900 $O/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread
tail -3 $O/pytest_gpu.log
grep -q " passed" $O/pytest_gpu.log && ! grep -q "failed" $O/pytest_gpu.log
$S 200 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
$S 200 $O/bench_bit.log python -u bench.py
$S 200 $O/bench_byte.log python -u bench.py --kernel byte --no-cpu-baseline
cat $O/bench_bit.log $O/bench_byte.log
export TMPDIR=/tmp
$S 200 $O/rp_bit.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bit -o run -- python3 bench.py --no-cpu-baseline
$S 200 $O/rp_byte.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_byte -o run -- python3 bench.py --kernel byte --no-cpu-baseline
