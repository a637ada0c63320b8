#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r1c; mkdir -p $O
S=scripts/gpu_step.sh
$S 600 $O/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tail -5 $O/pytest_gpu.log
$S 120 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
tail -2 $O/smoke.log
for m in torch_then_lib torch_cuda; do $S 120 $O/probe_$m.log python -u scripts/torch_probe.py $m; tail -2 $O/probe_$m.log; done
$S 240 $O/bench_bit.log python -u bench.py --kernel bit
tail -1 $O/bench_bit.log
$S 240 $O/bench_byte.log python -u bench.py --kernel byte --steps 30 --no-cpu-baseline
tail -1 $O/bench_byte.log
$S 240 $O/bench_p46.log python -u bench.py --workload p46gun_big --steps 10000 --warmup 10 --no-cpu-baseline
tail -1 $O/bench_p46.log
