#!/bin/bash
# r3f: tstep launch bound 6 waves/SIMD (byte tiles 92 -> 80 VGPRs, 3 per CU; spills only outside the generation
# loop): byte parity, A/B against HEAD's library (build_exp/head)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3f
mkdir -p $O
S=scripts/gpu_step.sh
H=$GRAFT_REPO_ROOT/build_exp/head/liblife_mi355x.so
$S 400 $O/pytest.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_golden.py -m gpu -x -q --timeout 200 --timeout-method thread -k "byte or temporal or split or c3 or c4" || exit $?
grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
for round in 1 2; do
  for v in head cur; do
    case $v in head) E="LIFE_MI355X_LIB=$H";; cur) E="LIFE_FLOW=1";; esac
    $S 200 $O/${v}_byte65536_$round.json env $E python -u bench.py --no-cpu-baseline --kernel byte --steps 480 --warmup 32 || exit $?
    $S 200 $O/${v}_byte32768_$round.json env $E python -u bench.py --no-cpu-baseline --kernel byte --size 32768 --steps 480 --warmup 32 || exit $?
    $S 200 $O/${v}_bitdriver_$round.json env $E python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 || exit $?
  done
done
