#!/bin/bash
# r5u: per-XCD queues for the dataflow tiles (LIFE_FLOW_XCD=1, experiment): flow parity suite with the
# queues on, then bench A/B at the default shape (generations 32..1024, where the dataflow form runs),
# 65536^2 and 32768^2, without / with the queues, and the per-launch tiles beside them.
# (The queues were 2-3 % slower and were removed after this job)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5u
rm -rf $O; mkdir -p $O
S=scripts/gpu_step.sh
LIFE_FLOW_XCD=1 $S 400 $O/pytest_flow_xcd.log python -u -m pytest tests/test_gpu_flow.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
tail -2 $O/pytest_flow_xcd.log; grep -q " passed" $O/pytest_flow_xcd.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest_flow_xcd.log || exit 1
for rep in 1 2; do
  for x in 0 1; do
    LIFE_FLOW_XCD=$x $S 200 $O/b65k_flow_x${x}_$rep.json python -u bench.py --flow 1 --no-cpu-baseline || exit $?
    LIFE_FLOW_XCD=$x $S 200 $O/b32k_flow_x${x}_$rep.json python -u bench.py --flow 1 --size 32768 --no-cpu-baseline || exit $?
  done
  $S 200 $O/b65k_tiles_$rep.json python -u bench.py --no-cpu-baseline || exit $?
  $S 200 $O/b32k_tiles_$rep.json python -u bench.py --size 32768 --no-cpu-baseline || exit $?
done
echo done
