#!/bin/bash
# VGPR-resident small-grid kernel: parity (small-grid, single-shard, p46 golden), configs[1] timing.
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1aa; mkdir -p $O
S=$R/scripts/gpu_step.sh
$S 300 $O/pytest_small.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -m gpu -x -q -k "small_grid or single_shard or p46gun" --timeout 120 --timeout-method thread
tail -4 $O/pytest_small.log
$S 200 $O/p46.log python -u scripts/p46_modes.py
cat $O/p46.log
$S 200 $O/bench_p46.log python -u bench.py --workload p46gun_big --steps 10000 --warmup 16 --no-cpu-baseline
grep '^{' $O/bench_p46.log | cut -c1-400
