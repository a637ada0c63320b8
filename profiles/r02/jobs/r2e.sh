#!/bin/bash
# r2e: GPU suite after the byte store fix; PMC passes on the bit sweep vs tiles
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r2e
mkdir -p $O
S=scripts/gpu_step.sh
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1
$S 900 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread || exit $?
B="python3 -u bench.py --no-cpu-baseline --steps 160 --warmup 16"
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_BUSY_CYCLES"
for v in sweep tiles; do
  extra=""; [ $v = tiles ] && extra="--temporal tiles"
  $S 120 $O/pmc1_$v.log timeout -s KILL 90 rocprofv3 --pmc $P1 --kernel-trace -d $O/pmc1_$v -o run -- $B $extra || exit $?
  $S 120 $O/pmc2_$v.log timeout -s KILL 90 rocprofv3 --pmc $P2 --kernel-trace -d $O/pmc2_$v -o run -- $B $extra || exit $?
done
