#!/bin/bash
# r04l: skewed tiles after the load-walk fix: parity test, A/B vs per-launch
# tiles (driver shape, default run), SQ counters of both on the driver shape.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r04/m; mkdir -p $O
S=scripts/gpu_step.sh
$S 600 $O/skew_test.log python -u -m pytest tests/test_gpu_parity.py -k "skewed or deep_halo" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/skew_test.log && ! grep -q -E "[0-9]+ (failed|error)" $O/skew_test.log || exit 1
i=0
for v in 0 1 1 0 0 1; do i=$((i+1)); LIFE_SKEW=$v $S 150 $O/drv_s${v}_$i.log python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?; done
i=0
for v in 1 0; do i=$((i+1)); LIFE_SKEW=$v $S 150 $O/def_s${v}_$i.log python -u bench.py --no-cpu-baseline || exit $?; done
cd /tmp && export TMPDIR=/tmp && cd $R
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
for v in 0 1; do
  LIFE_SKEW=$v $S 120 $O/pmc_s$v.log timeout -s KILL 100 rocprofv3 --pmc $A -d $O/pmc_s$v -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
done
LIFE_SKEW=1 $S 120 $O/trace_s1.log timeout -s KILL 100 rocprofv3 --kernel-trace --stats -d $O/trace_s1 -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
echo done
