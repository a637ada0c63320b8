#!/bin/bash
# r4j: SQ counter passes on the driver-shaped call (pair tiles) and on the in-register pair microbenchmark
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r4j; mkdir -p $O
R=$GRAFT_REPO_ROOT
S=scripts/gpu_step.sh
cd /tmp && export TMPDIR=/tmp && cd $R
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE"
B="SQ_ACTIVE_INST_VALU2 SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_LDS SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_SCA SQ_CYCLES GRBM_GUI_ACTIVE"
C="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
i=0
for P in "$A" "$B" "$C"; do i=$((i+1))
  $S 120 $O/tiles_$i.log timeout -s KILL 100 rocprofv3 --pmc $P -d $O/tiles_$i -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  $S 120 $O/ub_$i.log timeout -s KILL 100 rocprofv3 --pmc $P -d $O/ub_$i -o run --output-format csv -- $R/scripts/ubench_pair || exit $?
done
echo done
