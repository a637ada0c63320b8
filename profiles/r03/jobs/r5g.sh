#!/bin/bash
# r5g: parity at the working tree (one-generation XCD order on for bytes, one-ghost byte tiles for
# step(1)), the RCCL loopback bench line in rank mode without a launcher, one-generation and step(1) rates.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5g
mkdir -p $O
S=scripts/gpu_step.sh
$S 500 $O/pytest.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_rank.py tests/test_gpu_loopback.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider || exit $?
tail -2 $O/pytest.log; grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
$S 200 $O/bench_loop_rccl.json python -u bench.py --rank-mode --loopback --steps 20 --warmup 5 --no-cpu-baseline || exit $?
LIFE_TEMPORAL_DEPTH_BYTE=1 $S 200 $O/byte1.json python -u bench.py --kernel byte --steps 30 --warmup 10 --no-cpu-baseline || exit $?
$S 200 $O/step1.log python -u scripts/step1_rate.py || exit $?
for m in 7 8 10; do
  LIFE_BLOCK_GENS=$m $S 200 $O/drv_m$m.json python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
done
echo done
