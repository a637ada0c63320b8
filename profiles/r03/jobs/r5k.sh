#!/bin/bash
# r5k: byte one-generation default R16/D8 (XCD strip order): parity, bench lines, rocprofv3 stats.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5k
mkdir -p $O
S=scripts/gpu_step.sh
R=$GRAFT_REPO_ROOT
$S 500 $O/pytest.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q --timeout 250 --timeout-method thread -p no:cacheprovider || exit $?
tail -2 $O/pytest.log; grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
for i in 1 2; do
  LIFE_TEMPORAL_DEPTH_BYTE=1 $S 200 $O/byte1_$i.json python -u bench.py --kernel byte --steps 30 --warmup 10 --no-cpu-baseline || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd $R
LIFE_TEMPORAL_DEPTH_BYTE=1 $S 200 $O/rocprof_byte1.log rocprofv3 --kernel-trace --stats -d $O/prof_byte1 -o run --output-format csv -- python3 $R/bench.py --kernel byte --steps 30 --warmup 10 --no-cpu-baseline || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  LIFE_TEMPORAL_DEPTH_BYTE=1 $S 120 $O/pmc_$c.log timeout -s KILL 100 rocprofv3 --pmc $c -d $O/pmc_$c -o run --output-format csv -- python3 $R/bench.py --kernel byte --steps 30 --warmup 10 --no-cpu-baseline || exit $?
done
echo done
