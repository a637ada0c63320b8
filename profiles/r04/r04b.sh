#!/bin/bash
# r04b: GPU suite after the event-order fix; bit-tile stall attribution
# (timing-only variants: no barrier / no LDS permute / both) on the
# driver-shaped call; SQ counter passes; 8-LOCAL-shard host enqueue.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r04/b; mkdir -p $O
S=scripts/gpu_step.sh
$S 900 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
for i in 1 2; do
  $S 120 $O/v_base_$i.log python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  for v in nobar self both; do
    LIFE_MI355X_LIB=$R/build_exp/$v/liblife_mi355x.so $S 120 $O/v_${v}_$i.log python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  done
done
$S 300 $O/weak8.log python -u bench.py --gpus 8 --steps 20 --warmup 5 --no-cpu-baseline --no-parity || exit $?
$S 300 $O/strong8.log python -u bench.py --gpus 8 --scaling strong --steps 20 --warmup 5 --no-cpu-baseline --no-parity || exit $?
$S 300 $O/loop_rccl.log python -u bench.py --steps 20 --warmup 5 --rank-mode --loopback --no-cpu-baseline --no-parity || exit $?
cd /tmp && export TMPDIR=/tmp && cd $R
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
B="SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_CYCLES GRBM_GUI_ACTIVE"
i=0
for P in "$A" "$B"; do i=$((i+1))
  for v in base nobar; do
    if [ $v = base ]; then
      $S 120 $O/pmc_${v}_$i.log timeout -s KILL 100 rocprofv3 --pmc $P -d $O/pmc_${v}_$i -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
    else
      LIFE_MI355X_LIB=$R/build_exp/$v/liblife_mi355x.so $S 120 $O/pmc_${v}_$i.log timeout -s KILL 100 rocprofv3 --pmc $P -d $O/pmc_${v}_$i -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
    fi
  done
done
echo done
