#!/bin/bash
# Per-launch timing of the windowed small-grid kernel: small-grid/timing parity, p46 bench.
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1am; mkdir -p $O
S=$R/scripts/gpu_step.sh
$S 400 $O/pytest_small.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -m gpu -x -q -k "small or golden or p46 or cfg or timing" --timeout 120 --timeout-method thread
tail -3 $O/pytest_small.log
$S 200 $O/bench_p46.log python -u bench.py --workload p46gun_big --steps 10000 --warmup 64
cat $O/bench_p46.log
