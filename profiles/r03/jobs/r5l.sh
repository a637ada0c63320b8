#!/bin/bash
# r5l: byte tiles in strip-major order (LIFE_BYTE_STRIP = C tile columns per strip): parity with C = 8,
# A/B of C = 0 / 4 / 8 / 16 at 65536^2, FETCH_SIZE / WRITE_SIZE for C = 8.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5l
mkdir -p $O
S=scripts/gpu_step.sh
R=$GRAFT_REPO_ROOT
LIFE_BYTE_STRIP=8 $S 500 $O/pytest.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k byte -x -q --timeout 250 --timeout-method thread -p no:cacheprovider || exit $?
tail -2 $O/pytest.log; grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
for i in 1 2; do
  for c in 0 4 8 16; do
    LIFE_BYTE_STRIP=$c $S 200 $O/byte_c${c}_$i.json python -u bench.py --kernel byte --no-cpu-baseline || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp && cd $R
for c in 4 8; do
  for p in FETCH_SIZE WRITE_SIZE; do
    LIFE_BYTE_STRIP=$c $S 120 $O/pmc_c${c}_$p.log timeout -s KILL 100 rocprofv3 --pmc $p -d $O/pmc_c${c}_$p -o run --output-format csv -- python3 $R/bench.py --kernel byte --steps 64 --warmup 32 --no-cpu-baseline || exit $?
  done
done
echo done
