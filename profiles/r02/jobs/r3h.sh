#!/bin/bash
# r3h: right-neighbour ds_bpermute issued rows ahead of its use (build_exp/pref, a patched copy of HEAD): parity of the
# tile / flow paths under it, A/B against the tree's library
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3h
mkdir -p $O
S=scripts/gpu_step.sh
X=$GRAFT_REPO_ROOT/build_exp/pref/liblife_mi355x.so
$S 400 $O/pytest_pref.log env LIFE_MI355X_LIB=$X python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_parity.py tests/test_gpu_golden.py -m gpu -x -q --timeout 200 --timeout-method thread -k "flow or temporal or single_shard or multi_shard or golden or split" || exit $?
grep -q " passed" $O/pytest_pref.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest_pref.log || exit 1
for round in 1 2 3; do
  for v in tree pref; do
    case $v in tree) E="LIFE_FLOW=1";; pref) E="LIFE_MI355X_LIB=$X";; esac
    $S 200 $O/${v}_driver_$round.json env $E python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 || exit $?
    $S 200 $O/${v}_65536_$round.json env $E python -u bench.py --no-cpu-baseline --steps 480 --warmup 32 || exit $?
  done
done
