#!/bin/bash
# r04c: GPU suite with the deep halo + peer-only LOCAL ordering; loopback
# A/B deep on/off (20 and 992 generations); 8 LOCAL shards host enqueue;
# byte tile counters.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r04/c; mkdir -p $O
S=scripts/gpu_step.sh
$S 900 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
$S 120 $O/bench_driver.log python -u bench.py --steps 20 --warmup 5 || exit $?
for i in 1 2; do
  $S 120 $O/v_base_$i.log python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  LIFE_MI355X_LIB=$R/build_exp/reorder/liblife_mi355x.so $S 120 $O/v_reorder_$i.log python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  $S 120 $O/v_base992_$i.log python -u bench.py --no-cpu-baseline || exit $?
  LIFE_MI355X_LIB=$R/build_exp/reorder/liblife_mi355x.so $S 120 $O/v_reorder992_$i.log python -u bench.py --no-cpu-baseline || exit $?
done
LIFE_MI355X_LIB=$R/build_exp/reorder/liblife_mi355x.so $S 300 $O/reorder_parity.log python -u -m pytest tests/test_gpu_parity.py -k "temporal_single_shard or wide_periodic or deep_halo" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
for i in 1 2; do
  for dh in 1 0; do
    LIFE_DEEP_HALO=$dh $S 200 $O/loop20_d${dh}_$i.log python -u bench.py --steps 20 --warmup 5 --rank-mode --loopback --no-cpu-baseline --no-parity || exit $?
    LIFE_DEEP_HALO=$dh $S 200 $O/loop992_d${dh}_$i.log python -u bench.py --rank-mode --loopback --no-cpu-baseline --no-parity || exit $?
  done
done
LIFE_DEEP_HALO=1 $S 200 $O/loop20_serial.log python -u bench.py --steps 20 --warmup 5 --rank-mode --loopback --no-overlap --no-cpu-baseline --no-parity || exit $?
$S 300 $O/weak8.log python -u bench.py --gpus 8 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
$S 300 $O/strong8.log python -u bench.py --gpus 8 --scaling strong --steps 20 --warmup 5 --no-cpu-baseline || exit $?
$S 300 $O/strong4.log python -u bench.py --gpus 4 --scaling strong --steps 20 --warmup 5 --no-cpu-baseline || exit $?
$S 200 $O/byte.log python -u bench.py --kernel byte --steps 64 --warmup 32 --no-cpu-baseline || exit $?
cd /tmp && export TMPDIR=/tmp && cd $R
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
B="SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_VMEM SQ_CYCLES GRBM_GUI_ACTIVE"
i=0
for P in "$A" "$B"; do i=$((i+1))
  $S 120 $O/pmc_byte_$i.log timeout -s KILL 100 rocprofv3 --pmc $P -d $O/pmc_byte_$i -o run --output-format csv -- python3 $R/bench.py --kernel byte --steps 64 --warmup 32 --no-cpu-baseline || exit $?
done
echo done
