#!/bin/bash
# r04ag: rocprofv3 kernel trace + stats of the other bench lines (byte,
# RCCL loopback, 32768^2, p46gun_big) and the byte HBM passes, shipped build.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r04/ag; mkdir -p $O
S=scripts/gpu_step.sh
cd /tmp && export TMPDIR=/tmp && cd $R
$S 200 $O/trace_byte.log timeout -s KILL 190 rocprofv3 --kernel-trace --stats -d $O/trace_byte -o run --output-format csv -- python3 $R/bench.py --kernel byte --steps 64 --warmup 32 --no-cpu-baseline || exit $?
$S 150 $O/trace_loop20.log timeout -s KILL 140 rocprofv3 --kernel-trace --stats -d $O/trace_loop20 -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --rank-mode --loopback --no-cpu-baseline --no-parity || exit $?
$S 150 $O/trace_32768.log timeout -s KILL 140 rocprofv3 --kernel-trace --stats -d $O/trace_32768 -o run --output-format csv -- python3 $R/bench.py --size 32768 --no-cpu-baseline || exit $?
$S 150 $O/trace_p46.log timeout -s KILL 140 rocprofv3 --kernel-trace --stats -d $O/trace_p46 -o run --output-format csv -- python3 $R/bench.py --workload p46gun_big --no-cpu-baseline || exit $?
$S 120 $O/pmc_fetch_byte.log timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_byte -o run --output-format csv -- python3 $R/bench.py --kernel byte --steps 64 --warmup 32 --no-cpu-baseline || exit $?
$S 120 $O/pmc_write_byte.log timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_byte -o run --output-format csv -- python3 $R/bench.py --kernel byte --steps 64 --warmup 32 --no-cpu-baseline || exit $?
echo done
