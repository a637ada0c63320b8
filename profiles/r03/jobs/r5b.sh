#!/bin/bash
# r5b: parity at the working tree (XCD order on by default, masked extra-dword loads, depth-18
# strips); bit tiles with the neighbour ds_bpermute a row ahead behind a scheduling fence
# (build_exp/ahead2) vs the default; byte one-generation depth 18; byte tiles XCD order A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5b
mkdir -p $O
S=scripts/gpu_step.sh
R=$GRAFT_REPO_ROOT
A2=$R/build_exp/ahead2/liblife_mi355x.so
A1=$R/build_exp/ahead1/liblife_mi355x.so
$S 500 $O/pytest.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_flow.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider || exit $?
tail -2 $O/pytest.log; grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
LIFE_MI355X_LIB=$A2 $S 400 $O/pytest_a2.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider || exit $?
tail -2 $O/pytest_a2.log; grep -q " passed" $O/pytest_a2.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest_a2.log || exit 1
for i in 1 2 3; do
  $S 200 $O/drv_main_$i.json python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  LIFE_MI355X_LIB=$A2 $S 200 $O/drv_a2_$i.json python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  LIFE_MI355X_LIB=$A1 $S 200 $O/drv_a1_$i.json python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
done
for i in 1 2; do
  $S 200 $O/def_main_$i.json python -u bench.py --no-cpu-baseline || exit $?
  LIFE_MI355X_LIB=$A2 $S 200 $O/def_a2_$i.json python -u bench.py --no-cpu-baseline || exit $?
  LIFE_MI355X_LIB=$A1 $S 200 $O/def_a1_$i.json python -u bench.py --no-cpu-baseline || exit $?
done
LIFE_TEMPORAL_DEPTH_BYTE=1 $S 300 $O/tune_byte1.log python -u scripts/tune.py --kernels byte --rows 16,64 --depths 2,8,18 --gens 10 --rounds 3 || exit $?
LIFE_TEMPORAL_DEPTH=1 $S 300 $O/tune_bit1.log python -u scripts/tune.py --kernels bit --rows 16 --depths 8,18 --gens 10 --rounds 3 || exit $?
for i in 1 2; do
  for x in 0 1; do
    LIFE_XCD_ORDER_BYTE=$x $S 200 $O/byte_x${x}_$i.json python -u bench.py --kernel byte --no-cpu-baseline || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp && cd $R
for c in FETCH_SIZE WRITE_SIZE; do
  LIFE_XCD_ORDER_BYTE=1 $S 120 $O/pmc_bytex1_$c.log timeout -s KILL 100 rocprofv3 --pmc $c -d $O/pmc_bytex1_$c -o run --output-format csv -- python3 $R/bench.py --kernel byte --steps 64 --warmup 32 --no-cpu-baseline || exit $?
done
echo done
