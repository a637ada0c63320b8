#!/bin/bash
# r05m: SQ counters of the dataflow form against the per-launch tiles at
# 32768^2 (96 generations): where a dataflow item's extra ~20 % of body time
# goes (r05c traces) now that its permutes are issued ahead (r05j) -- more
# waves waiting (SQ_WAIT_ANY: barriers / polls), fewer VALU issued per busy
# cycle, or more instructions (SALU / SMEM / LDS per item).
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r05/m; mkdir -p $O
S=scripts/gpu_step.sh
cd /tmp && export TMPDIR=/tmp && cd $R
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS"
for f in 0 1; do
  $S 120 $O/pmc1_f$f.log timeout -s KILL 100 rocprofv3 --pmc $P1 -d $O/pmc1_f$f -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --shape 32768x32768 --steps 96 --warmup 32 --flow $f || exit $?
  $S 120 $O/pmc2_f$f.log timeout -s KILL 100 rocprofv3 --pmc $P2 -d $O/pmc2_f$f -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --shape 32768x32768 --steps 96 --warmup 32 --flow $f || exit $?
done
echo done
