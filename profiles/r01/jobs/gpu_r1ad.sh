#!/bin/bash
# Bench lines with the live copy ceiling; rocprof stats of the default bench.
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1ad; mkdir -p $O
S=$R/scripts/gpu_step.sh
$S 200 $O/pytest_copy.log python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "copy or small_grid" --timeout 120 --timeout-method thread
tail -1 $O/pytest_copy.log
$S 240 $O/bench_bit.log python -u bench.py
grep '^{' $O/bench_bit.log | cut -c1-200
$S 240 $O/bench_byte.log python -u bench.py --kernel byte --no-cpu-baseline
$S 240 $O/bench_bit_onegen.log env LIFE_TEMPORAL_DEPTH=1 python -u bench.py --no-cpu-baseline --steps 64
$S 240 $O/bench_p46.log python -u bench.py --workload p46gun_big --steps 10000 --warmup 16 --no-cpu-baseline
cd /tmp && export TMPDIR=/tmp
$S 300 $O/rocprof_bit.log rocprofv3 --kernel-trace --stats -d $O/prof_bit -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline
$S 300 $O/rocprof_p46.log rocprofv3 --kernel-trace --stats -d $O/prof_p46 -o run --output-format csv -- python3 $R/bench.py --workload p46gun_big --steps 10000 --warmup 16 --no-cpu-baseline
ls $O/prof_p46
