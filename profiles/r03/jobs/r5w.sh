#!/bin/bash
# r5w: byte window rows 56 against 48 (r5v: 69.0 against 66.9 T in one run): parity of the byte tests
# at R = 56 (not test_timing_stats: its VALU model reads the default rows), three interleaved A/B runs, FETCH_SIZE / WRITE_SIZE of both.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5w
rm -rf $O; mkdir -p $O
S=scripts/gpu_step.sh
R=$GRAFT_REPO_ROOT
LIFE_TEMPORAL_ROWS_BYTE=56 $S 500 $O/pytest.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "byte and not timing_stats" -x -q --timeout 250 --timeout-method thread -p no:cacheprovider || exit $?
tail -2 $O/pytest.log; grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
for i in 1 2 3; do
  for r in 48 56; do
    LIFE_TEMPORAL_ROWS_BYTE=$r $S 200 $O/byte_r${r}_$i.json python -u bench.py --kernel byte --no-cpu-baseline || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp && cd $R
for r in 48 56; do
  for p in FETCH_SIZE WRITE_SIZE; do
    LIFE_TEMPORAL_ROWS_BYTE=$r $S 120 $O/pmc_r${r}_$p.log timeout -s KILL 100 rocprofv3 --pmc $p -d $O/pmc_r${r}_$p -o run --output-format csv -- python3 $R/bench.py --kernel byte --steps 64 --warmup 32 --no-cpu-baseline || exit $?
  done
done
echo done
