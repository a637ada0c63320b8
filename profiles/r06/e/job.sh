#!/bin/bash
# r06e: validation of the round-6 product.  Smoke; the whole GPU suite (with
# the new whole-grid 65536^2 oracle check and the 1-1.5-round flow rule);
# the bench lines DESIGN 5.5 quotes; the 16384x32768 pass traced with HEAD's
# banded half-height tail and with the round-4 library's unbanded one (same
# box).  Expectation: all green; driver line ~100-102 T (0.45 of VALU);
# 16384x32768 auto -> tiles ~83 T (r4: ~72 T).
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r06/e; mkdir -p $O
S=scripts/gpu_step.sh
T="python -u -m pytest -x -q --timeout 600 --timeout-method thread -p no:cacheprovider"
$S 120 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
$S 200 $O/bench_driver.log python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
U="python -u bench.py --no-cpu-baseline"
$S 150 $O/bench_driver2.log $U --gpus 1 --steps 20 --warmup 5 || exit $?
$S 150 $O/bench_default.log $U || exit $?
$S 150 $O/c2_32768.log $U --shape 32768x32768 || exit $?
$S 150 $O/c2_32768_byte.log $U --shape 32768x32768 --kernel byte || exit $?
$S 150 $O/c1_p46.log $U --workload p46gun_big || exit $?
$S 200 $O/bench_byte.log $U --kernel byte || exit $?
$S 150 $O/u16384x32768.log $U --shape 16384x32768 || exit $?
$S 300 $O/rehearse8.log $U --gpus 8 --rehearse-shards --steps 20 --warmup 5 || exit $?
$S 150 $O/loop20_65536.log $U --rank-mode --loopback --no-parity --steps 20 --warmup 5 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $R
$S 150 $O/trace_16384.log timeout -s KILL 140 rocprofv3 --kernel-trace --stats -d $O/trace_16384 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --shape 16384x32768 --steps 96 --warmup 32 || exit $?
LIFE_MI355X_LIB=$R/build_exp/r4/liblife_mi355x.so $S 150 $O/trace_16384_r4.log timeout -s KILL 140 rocprofv3 --kernel-trace --stats -d $O/trace_16384_r4 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --shape 16384x32768 --flow 0 --steps 96 --warmup 32 || exit $?
$S 1150 $O/pytest.log $T tests -m gpu || exit $?
grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
echo done
