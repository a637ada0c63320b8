#!/bin/bash
# Drifting-frame temporal kernel: temporal parity, full-size parity, bench bit and byte.
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1ao; mkdir -p $O
S=$R/scripts/gpu_step.sh
$S 300 $O/pytest_temporal.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "temporal or timing or multi_shard" --timeout 120 --timeout-method thread
tail -3 $O/pytest_temporal.log
grep -q " passed" $O/pytest_temporal.log && ! grep -q "failed" $O/pytest_temporal.log
$S 200 $O/bench_bit.log python -u bench.py --no-cpu-baseline
cat $O/bench_bit.log
$S 200 $O/bench_byte.log python -u bench.py --kernel byte --no-cpu-baseline
cat $O/bench_byte.log
$S 400 $O/pytest_full.log python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -q --timeout 240 --timeout-method thread
tail -3 $O/pytest_full.log
