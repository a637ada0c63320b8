#!/bin/bash
# Windowed small-grid kernel with DPP row rotates, automatic K = 30: full GPU suite, p46 bench + rocprof stats, default bench.
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1al; mkdir -p $O
S=$R/scripts/gpu_step.sh
$S 900 $O/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread
tail -3 $O/pytest_gpu.log
$S 200 $O/bench_p46.log python -u bench.py --workload p46gun_big --steps 10000 --warmup 64
cat $O/bench_p46.log
export TMPDIR=/tmp
$S 300 $O/rocprof_p46.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_p46 -o run -- python3 bench.py --workload p46gun_big --steps 10000 --warmup 64 --no-cpu-baseline
tail -2 $O/rocprof_p46.log
$S 300 $O/bench.log python -u bench.py
cat $O/bench.log
