#!/bin/bash
# r3b: (1) tail split generalised to a full-width interior region (row strips): tests + 2-shard A/B;
# (2) banded last column inside the dataflow kernel through a non-inlined call (build_exp/flowband, a patched copy of
# 8178773's csrc): flow parity/census, A/B against the tree's library
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3b
mkdir -p $O
S=scripts/gpu_step.sh
X=$GRAFT_REPO_ROOT/build_exp/flowband/liblife_mi355x.so
$S 400 $O/pytest_split.log python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_loopback.py -m gpu -x -q --timeout 200 --timeout-method thread -k "split or temporal or multi_shard or loopback" || exit $?
grep -q " passed" $O/pytest_split.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest_split.log || exit 1
$S 300 $O/pytest_flowband.log env LIFE_MI355X_LIB=$X python -u -m pytest tests/test_gpu_flow.py -m gpu -x -q --timeout 200 --timeout-method thread -k "parity or census" || exit $?
grep -q " passed" $O/pytest_flowband.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest_flowband.log || exit 1
for round in 1 2; do
  for sp in 0 1; do
    $S 200 $O/strips2_s${sp}_$round.json env LIFE_TAIL_SPLIT=$sp python -u bench.py --gpus 2 --no-cpu-baseline --no-parity --steps 20 --warmup 5 || exit $?
  done
  for v in head band; do
    case $v in head) E="LIFE_FLOW=1";; band) E="LIFE_MI355X_LIB=$X";; esac
    $S 200 $O/${v}_65536_$round.json env $E python -u bench.py --no-cpu-baseline --steps 480 --warmup 32 || exit $?
    $S 200 $O/${v}_16384_$round.json env $E python -u bench.py --no-cpu-baseline --size 16384 --steps 960 --warmup 32 || exit $?
  done
done
