#!/bin/bash
# r4d: repeated pass-size points for the two bench shapes (pair tiles 24x8, 24x12), then
# a kernel + HIP API trace of the driver-shaped call at m = 12 (host gap)
O=gpurun_out/r4d; mkdir -p $O
timeout -k 10 400 python scripts/shape_sweep.py $O/sweep.jsonl --shapes 24x8 --m 8,10,12,20 --modes driver --reps 3 &&
timeout -k 10 400 python scripts/shape_sweep.py $O/sweep.jsonl --shapes 24x8 --m 12,14,16 --modes default --reps 2 &&
timeout -k 10 300 python scripts/shape_sweep.py $O/sweep.jsonl --shapes 24x12 --m 16,20 --modes default,driver --reps 2 &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
LIFE_BLOCK_GENS=12 timeout -k 10 120 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $O/trace -o drv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/trace_bench.json 2> $O/trace.err; tail -2 $O/trace.err; ls -R $O/trace | head
