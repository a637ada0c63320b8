#!/bin/bash
# r06m: the round's closing profile of the driver-shaped command on the
# final library: rocprofv3 kernel trace + stats (the tstep_bit_kernel average
# must agree with the bench line's kernel_avg_ms), then the FETCH_SIZE and
# WRITE_SIZE passes (one counter block per run).
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r06/m; mkdir -p $O
S=scripts/gpu_step.sh
cd /tmp && export TMPDIR=/tmp && cd $R
$S 150 $O/trace_driver.log timeout -s KILL 140 rocprofv3 --kernel-trace --stats -d $O/trace_driver -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
$S 100 $O/pmc_fetch.log timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
$S 100 $O/pmc_write.log timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
echo done
