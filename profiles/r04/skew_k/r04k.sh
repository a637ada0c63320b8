#!/bin/bash
# r04k: skewed (ghost-free) bit tiles: parity (the new test, then the
# temporal / golden / deep-halo suites with LIFE_SKEW=1), then A/B against
# the per-launch tiles on the driver shape and the default run.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r04/k; mkdir -p $O
S=scripts/gpu_step.sh
$S 600 $O/skew_test.log python -u -m pytest tests/test_gpu_parity.py -k skewed -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/skew_test.log && ! grep -q -E "[0-9]+ (failed|error)" $O/skew_test.log || exit 1
LIFE_SKEW=1 $S 900 $O/skew_suite.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_loopback.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "not timing_stats and not exchange_count" || exit $?
i=0
for v in 0 1 1 0 0 1; do i=$((i+1)); LIFE_SKEW=$v $S 150 $O/drv_s${v}_$i.log python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?; done
i=0
for v in 0 1 1 0; do i=$((i+1)); LIFE_SKEW=$v $S 150 $O/def_s${v}_$i.log python -u bench.py --no-cpu-baseline || exit $?; done
LIFE_SKEW=1 $S 150 $O/loop20_s1.log python -u bench.py --steps 20 --warmup 5 --rank-mode --loopback --no-cpu-baseline --no-parity || exit $?
LIFE_SKEW=1 $S 150 $O/c2_s1.log python -u bench.py --size 32768 --no-cpu-baseline || exit $?
echo done
