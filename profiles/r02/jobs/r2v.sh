#!/bin/bash
# r2v: device-packed bits frames (gather_bits tests, frames at scale), stream priorities A/B on the partitioned
# 20-generation call (loopback LOCAL / RCCL, RCCL barrier in rank mode), golden driver tests
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2v
mkdir -p $O
S=scripts/gpu_step.sh
$S 400 $O/pytest.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_loopback.py tests/test_gpu_rank.py tests/test_gpu_bench.py -m gpu -x -q --timeout 200 --timeout-method thread -k "gather_bits or golden or driver or loopback or rank or bench or frames or resume" || exit $?
grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
for pr in 1 0; do
  $S 200 $O/loop_local_pr$pr.json env LIFE_STREAM_PRIORITY=$pr python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --loopback || exit $?
  $S 200 $O/loop_rccl_pr$pr.json env LIFE_STREAM_PRIORITY=$pr python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2955$pr bench.py --rank-mode --loopback --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  $S 200 $O/loop_rccl_long_pr$pr.json env LIFE_STREAM_PRIORITY=$pr python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2956$pr bench.py --rank-mode --loopback --steps 480 --warmup 32 --no-cpu-baseline || exit $?
done
$S 200 $O/driver_w5.json python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 || exit $?
$S 600 $O/frames.json python -u scripts/frames_at_scale.py --n 32768 --gens 1000 --save 100 --dir /dev/shm || exit $?
