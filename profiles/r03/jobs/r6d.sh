#!/bin/bash
# r6d: timing mode 2 (launches stamped by their dispatches, no phase events) for bench.py's timed call
# on partitioned steps: loopback / multi-shard parity and the new timing-mode test, then A/B of the
# bench lines with the phase events inside (LIFE_BENCH_PHASES_TIMED=1, the old form) and outside the
# timed call; a kernel trace of the new form.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6d
rm -rf $O; mkdir -p $O
S=scripts/gpu_step.sh
R=$GRAFT_REPO_ROOT
$S 500 $O/pytest.log python -u -m pytest tests/test_gpu_bench.py tests/test_gpu_parity.py tests/test_gpu_loopback.py tests/test_gpu_rank.py -k "multi_shard or loopback or rank or bench" -x -q --timeout 250 --timeout-method thread -p no:cacheprovider || exit $?
tail -2 $O/pytest.log; grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
for i in 1 2; do
  for t in 1 0; do
    LIFE_BENCH_PHASES_TIMED=$t $S 200 $O/rccl20_t${t}_$i.json python -u bench.py --rank-mode --loopback --steps 20 --warmup 5 --no-cpu-baseline || exit $?
    LIFE_BENCH_PHASES_TIMED=$t $S 200 $O/rccl992_t${t}_$i.json python -u bench.py --rank-mode --loopback --no-cpu-baseline || exit $?
    LIFE_BENCH_PHASES_TIMED=$t $S 200 $O/local20_t${t}_$i.json python -u bench.py --loopback --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  done
done
$S 200 $O/drv.json python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
cd /tmp && export TMPDIR=/tmp && cd $R
$S 200 $O/trace.log rocprofv3 --kernel-trace -d $O/trace_t0 -o run --output-format csv -- python3 $R/bench.py --rank-mode --loopback --steps 20 --warmup 5 --no-cpu-baseline || exit $?
echo done
