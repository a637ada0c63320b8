#!/bin/bash
# r04x: host enqueue cost per runtime call (scripts/ubench_enqueue.hip) and
# the LOCAL strong-8 / weak-8 call diagnostics on the same box.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04/x; mkdir -p $O
S=scripts/gpu_step.sh
$S 60 $O/ubench_enqueue.log scripts/ubench_enqueue || exit $?
$S 300 $O/strong8.log python -u bench.py --gpus 8 --scaling strong --steps 20 --warmup 5 --no-cpu-baseline || exit $?
$S 300 $O/weak8.log python -u bench.py --gpus 8 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
echo done
