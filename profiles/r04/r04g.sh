#!/bin/bash
# r04g: ABBA order A/B (this build vs r4b) on the driver shape; rocprofv3
# kernel trace + stats of the driver-shaped bench call and of the default run.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r04/g; mkdir -p $O
S=scripts/gpu_step.sh
B="LIFE_MI355X_LIB=$R/build_exp/r4b/liblife_mi355x.so"
i=0
for v in cur r4b r4b cur cur r4b r4b cur; do i=$((i+1))
  if [ $v = cur ]; then
    $S 120 $O/${v}_$i.log python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  else
    LIFE_MI355X_LIB=$R/build_exp/r4b/liblife_mi355x.so $S 120 $O/${v}_$i.log python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  fi
done
cd /tmp && export TMPDIR=/tmp && cd $R
$S 150 $O/trace_driver.log timeout -s KILL 140 rocprofv3 --kernel-trace --stats -d $O/trace_driver -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
$S 200 $O/trace_default.log timeout -s KILL 190 rocprofv3 --kernel-trace --stats -d $O/trace_default -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline || exit $?
$S 200 $O/trace_loop20.log timeout -s KILL 190 rocprofv3 --kernel-trace --stats -d $O/trace_loop20 -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --rank-mode --loopback --no-cpu-baseline --no-parity || exit $?
echo done
