#!/bin/bash
# Bench at the new defaults (warmup 960, steps 960): bit with cpu_baseline, byte; rocprof stats and trace of both.
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1as; mkdir -p $O
S=$R/scripts/gpu_step.sh
$S 200 $O/bench_bit.log python -u bench.py
cat $O/bench_bit.log
$S 200 $O/bench_byte.log python -u bench.py --kernel byte --no-cpu-baseline
cat $O/bench_byte.log
export TMPDIR=/tmp
$S 200 $O/rp_bit.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bit -o run -- python3 bench.py --no-cpu-baseline
$S 200 $O/rp_byte.log rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_byte -o run -- python3 bench.py --kernel byte --no-cpu-baseline
