#!/bin/bash
# r05u: why the dataflow form ran the driver's 2-pass call at 0.565 ms per
# pass (r05r) when its long runs at 65536^2 take ~0.45: a fixed cost per
# persistent launch should fall as 1/passes.  2, 4, 8 and 16 passes of 10
# generations in one launch (65536^2), hand-off forms 1 and 2, and a
# rocprofv3 kernel trace of the 2-pass call.  Expectation: per-pass time
# ~0.45 + C/passes with C ~0.25 ms (a per-launch cost to find), or flat
# ~0.56 (then the items themselves are slow at m = 10).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/u; mkdir -p $O
S=scripts/gpu_step.sh
for n in 2 4 8 16; do
  st=$((10 * n))
  LIFE_FLOW_MIN_PASSES=2 LIFE_BLOCK_GENS=10 $S 120 $O/flow1_p$n.log python -u bench.py --gpus 1 --steps $st --warmup 5 --no-cpu-baseline --flow 1 || exit $?
done
LIFE_FLOW_MIN_PASSES=2 LIFE_BLOCK_GENS=10 $S 120 $O/flow2_p2.log python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --flow 2 || exit $?
LIFE_FLOW_MIN_PASSES=2 LIFE_BLOCK_GENS=10 $S 120 $O/flow2_p8.log python -u bench.py --gpus 1 --steps 80 --warmup 5 --no-cpu-baseline --flow 2 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
LIFE_FLOW_MIN_PASSES=2 LIFE_BLOCK_GENS=10 $S 150 $O/trace_p2.log timeout -s KILL 140 rocprofv3 --kernel-trace -d $O/trace_p2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --flow 1 || exit $?
echo done
