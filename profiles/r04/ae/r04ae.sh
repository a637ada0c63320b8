#!/bin/bash
# r04ae: validation of the round-4 product (fast wrap on): smoke, the GPU suite, the bench
# lines, rocprofv3 kernel trace + stats of the driver-shaped command and the
# default run, FETCH/WRITE PMC passes of the driver-shaped call.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r04/ae; mkdir -p $O
S=scripts/gpu_step.sh
$S 120 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
$S 900 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
$S 200 $O/bench_driver.log python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
$S 200 $O/bench_default.log python -u bench.py --no-cpu-baseline || exit $?
$S 200 $O/loop20.log python -u bench.py --steps 20 --warmup 5 --rank-mode --loopback --no-cpu-baseline --no-parity || exit $?
$S 300 $O/weak8.log python -u bench.py --gpus 8 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
LIFE_SKEW=1 $S 300 $O/skew_suite.log python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
$S 200 $O/bench_byte.log python -u bench.py --kernel byte --no-cpu-baseline || exit $?
cd /tmp && export TMPDIR=/tmp && cd $R
$S 150 $O/trace_driver.log timeout -s KILL 140 rocprofv3 --kernel-trace --stats -d $O/trace_driver -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
$S 200 $O/trace_default.log timeout -s KILL 190 rocprofv3 --kernel-trace --stats -d $O/trace_default -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline || exit $?
$S 90 $O/pmc_fetch.log timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
$S 90 $O/pmc_write.log timeout -s KILL 80 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
echo done
