#!/bin/bash
# r04s: counters of the per-launch tiles (in-tree build) against the skewed
# segments with falling priority (build_exp/p3): HBM bytes (FETCH_SIZE x2 /
# WRITE_SIZE, one pass each), L2 hits and misses, LDS instructions, waits and
# bank conflicts.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r04/s; mkdir -p $O
S=scripts/gpu_step.sh
cd /tmp && export TMPDIR=/tmp && cd $R
P1="FETCH_SIZE"
P2="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
P3="SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE"
for v in base p3; do
  if [ $v = base ]; then export LIFE_SKEW=0; unset LIFE_MI355X_LIB; else export LIFE_SKEW=1 LIFE_MI355X_LIB=$R/build_exp/p3/liblife_mi355x.so; fi
  k=0
  for P in "$P1" "$P2" "$P3"; do k=$((k+1))
    $S 90 $O/pmc${k}_$v.log timeout -s KILL 80 rocprofv3 --pmc $P -d $O/pmc${k}_$v -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  done
done
echo done
