#!/bin/bash
# r04n: skewed tiles at exactly 40 KB of LDS: parity subset + driver A/B.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r04/n; mkdir -p $O
S=scripts/gpu_step.sh
$S 600 $O/skew_test.log python -u -m pytest tests/test_gpu_parity.py -k "skewed" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/skew_test.log && ! grep -q -E "[0-9]+ (failed|error)" $O/skew_test.log || exit 1
i=0
for v in 1 0 0 1; do i=$((i+1)); LIFE_SKEW=$v $S 150 $O/drv_s${v}_$i.log python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?; done
cd /tmp && export TMPDIR=/tmp && cd $R
LIFE_SKEW=1 $S 120 $O/trace_s1.log timeout -s KILL 100 rocprofv3 --kernel-trace -d $O/trace_s1 -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
echo done
