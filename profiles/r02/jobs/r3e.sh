#!/bin/bash
# r3e: no entry fence for single-stream step calls: parity subset, A/B (wall - kernel gap of the 20-generation call)
# against HEAD's library (build_exp/head)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3e
mkdir -p $O
S=scripts/gpu_step.sh
H=$GRAFT_REPO_ROOT/build_exp/head/liblife_mi355x.so
$S 400 $O/pytest.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_flow.py -m gpu -x -q --timeout 200 --timeout-method thread || exit $?
grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
for round in 1 2 3; do
  for v in head cur; do
    case $v in head) E="LIFE_MI355X_LIB=$H";; cur) E="LIFE_FLOW=1";; esac
    $S 200 $O/${v}_driver_$round.json env $E python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 || exit $?
  done
done
