#!/bin/bash
# r2i: bench --scaling strong|weak self-checks (parity_vs_1gpu, phases)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2i
mkdir -p $O
S=scripts/gpu_step.sh
$S 600 $O/pytest_bench.log python -u -m pytest tests/test_gpu_bench.py -x -v --timeout 300 --timeout-method thread || exit $?
$S 300 $O/strong4.json python -u bench.py --gpus 4 --scaling strong --steps 64 --warmup 16 --no-cpu-baseline || exit $?
$S 300 $O/weak2.json python -u bench.py --gpus 2 --steps 64 --warmup 16 --no-cpu-baseline || exit $?
