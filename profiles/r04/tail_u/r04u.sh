#!/bin/bash
# r04u: the per-launch tiles' tail -- half-height tail tiles whatever the
# last round's fill (LIFE_TAIL_MODE=1) against the default (split only when
# the last round is under half full), with workgroup timelines of both.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04/u; mkdir -p $O
S=scripts/gpu_step.sh
B="python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline"
LIFE_TAIL_MODE=1 $S 120 $O/test_t1.log python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py || exit $?
for t in 0 1; do LIFE_MI355X_LIB=build_exp/trc/liblife_mi355x.so LIFE_TAIL_MODE=$t $S 120 $O/trace_t$t.log python -u scripts/wg_trace.py 20 $O/trace_t$t.npy || exit $?; done
for i in 1 2 3; do
  for t in 0 1; do LIFE_TAIL_MODE=$t $S 150 $O/t${t}_$i.log $B || exit $?; done
done
for t in 0 1; do LIFE_TAIL_MODE=$t $S 200 $O/def_t$t.log python -u bench.py --no-cpu-baseline || exit $?; done
echo done
