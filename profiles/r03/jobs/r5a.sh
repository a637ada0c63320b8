#!/bin/bash
# r5a: XCD-aware bit tile order A/B (LIFE_XCD_ORDER 0/1: time + FETCH/WRITE), one-generation
# kernels with the extra-dword load masked to lanes 0/63 (A/B against HEAD's build), 32768^2
# dataflow vs per-launch tiles.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5a
mkdir -p $O
S=scripts/gpu_step.sh
R=$GRAFT_REPO_ROOT
BASE=$R/build_exp/base/liblife_mi355x.so
$S 400 $O/pytest_parity.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
tail -2 $O/pytest_parity.log; grep -q " passed" $O/pytest_parity.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest_parity.log || exit 1
for i in 1 2; do
  for x in 0 1; do
    LIFE_XCD_ORDER=$x $S 200 $O/drv_x${x}_$i.json python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
    LIFE_XCD_ORDER=$x $S 200 $O/def_x${x}_$i.json python -u bench.py --no-cpu-baseline || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp && cd $R
for c in FETCH_SIZE WRITE_SIZE; do
  LIFE_XCD_ORDER=1 $S 120 $O/pmc_x1_$c.log timeout -s KILL 100 rocprofv3 --pmc $c -d $O/pmc_x1_$c -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
done
for i in 1 2; do
  LIFE_TEMPORAL_DEPTH_BYTE=1 LIFE_MI355X_LIB=$BASE $S 200 $O/byte1_base_$i.json python -u bench.py --kernel byte --steps 30 --warmup 10 --no-cpu-baseline || exit $?
  LIFE_TEMPORAL_DEPTH_BYTE=1 $S 200 $O/byte1_new_$i.json python -u bench.py --kernel byte --steps 30 --warmup 10 --no-cpu-baseline || exit $?
  LIFE_TEMPORAL_DEPTH=1 LIFE_MI355X_LIB=$BASE $S 200 $O/bit1_base_$i.json python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline || exit $?
  LIFE_TEMPORAL_DEPTH=1 $S 200 $O/bit1_new_$i.json python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline || exit $?
done
LIFE_TEMPORAL_DEPTH_BYTE=1 $S 300 $O/tune_byte1.log python -u scripts/tune.py --kernels byte --rows 16,32,64 --depths 2,4,8 --gens 10 --rounds 3 || exit $?
for f in 0 1; do
  $S 200 $O/s32768_flow$f.json python -u bench.py --size 32768 --flow $f --no-cpu-baseline || exit $?
done
echo done
