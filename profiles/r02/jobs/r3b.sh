#!/bin/bash
# r3b: banded last column inside the dataflow kernel through a non-inlined call (build_exp/flowband, built from a
# patched copy of HEAD's csrc): flow parity/census, A/B against HEAD
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3b
mkdir -p $O
S=scripts/gpu_step.sh
X=$GRAFT_REPO_ROOT/build_exp/flowband/liblife_mi355x.so
$S 300 $O/pytest_flowband.log env LIFE_MI355X_LIB=$X python -u -m pytest tests/test_gpu_flow.py -m gpu -x -q --timeout 200 --timeout-method thread || exit $?
grep -q " passed" $O/pytest_flowband.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest_flowband.log || exit 1
for round in 1 2 3; do
  for v in head band; do
    case $v in head) E="LIFE_FLOW=1";; band) E="LIFE_MI355X_LIB=$X";; esac
    $S 200 $O/${v}_65536_$round.json env $E python -u bench.py --no-cpu-baseline --steps 480 --warmup 32 || exit $?
    $S 200 $O/${v}_16384_$round.json env $E python -u bench.py --no-cpu-baseline --size 16384 --steps 960 --warmup 32 || exit $?
  done
done
