#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r1h; mkdir -p $O
S=scripts/gpu_step.sh
$S 700 $O/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tail -4 $O/pytest_gpu.log
$S 120 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
tail -1 $O/smoke.log
$S 240 $O/bench_bit.log python -u bench.py --kernel bit
grep '^{' $O/bench_bit.log | cut -c1-200
$S 240 $O/bench_p46.log python -u bench.py --workload p46gun_big --steps 10000 --warmup 10 --no-cpu-baseline
grep '^{' $O/bench_p46.log | cut -c1-200
$S 240 $O/bench_p46_byte.log python -u bench.py --workload p46gun_big --kernel byte --steps 10000 --warmup 10 --no-cpu-baseline
grep '^{' $O/bench_p46_byte.log | cut -c1-200
