#!/bin/bash
# r5r: kernel traces of the RCCL loopback schedule, serial and overlapped (where the halo time goes).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5r
mkdir -p $O
S=scripts/gpu_step.sh
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $R
$S 200 $O/serial.log rocprofv3 --kernel-trace -d $O/trace_serial -o run --output-format csv -- python3 $R/bench.py --rank-mode --loopback --no-overlap --steps 20 --warmup 5 --no-cpu-baseline || exit $?
$S 200 $O/overlap.log rocprofv3 --kernel-trace -d $O/trace_overlap -o run --output-format csv -- python3 $R/bench.py --rank-mode --loopback --steps 20 --warmup 5 --no-cpu-baseline || exit $?
echo done
