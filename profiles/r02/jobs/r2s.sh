#!/bin/bash
# r2s: re-validation after container rebuild (flow default): full GPU suite, smoke, bench lines, rocprofv3 kernel stats of the default bench
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2s
mkdir -p $O
S=scripts/gpu_step.sh
R=$GRAFT_REPO_ROOT
$S 600 $O/pytest.log python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread || exit $?
grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
$S 300 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
$S 300 $O/bench_default.json python -u bench.py || exit $?
$S 300 $O/bench_byte.json python -u bench.py --kernel byte --no-cpu-baseline || exit $?
$S 300 $O/bench_32768.json python -u bench.py --size 32768 --no-cpu-baseline || exit $?
$S 300 $O/bench_32768_byte.json python -u bench.py --size 32768 --kernel byte --no-cpu-baseline || exit $?
$S 300 $O/bench_driver.json python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
$S 300 $O/bench_p46.json python -u bench.py --workload p46gun_big --steps 10000 --warmup 16 --no-cpu-baseline || exit $?
$S 300 $O/rocprof_bit.log rocprofv3 --kernel-trace --stats -d $O/prof_bit -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline || exit $?
