#!/bin/bash
# r04e: same-box A/B of the driver-shaped bit call: this build vs the
# round-3 product (ae5d1e6) vs r04b's build (73155f3); clock from PMC.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r04/e; mkdir -p $O
S=scripts/gpu_step.sh
for i in 1 2 3; do
  $S 120 $O/cur_$i.log python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  for v in r3 r4b; do
    LIFE_MI355X_LIB=$R/build_exp/$v/liblife_mi355x.so $S 120 $O/${v}_$i.log python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp && cd $R
P="SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT"
$S 120 $O/pmc_cur.log timeout -s KILL 100 rocprofv3 --pmc $P -d $O/pmc_cur -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
LIFE_MI355X_LIB=$R/build_exp/r3/liblife_mi355x.so $S 120 $O/pmc_r3.log timeout -s KILL 100 rocprofv3 --pmc $P -d $O/pmc_r3 -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
$S 120 $O/trace_cur.log timeout -s KILL 100 rocprofv3 --kernel-trace --stats -d $O/trace_cur -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
echo done
