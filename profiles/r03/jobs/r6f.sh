#!/bin/bash
# r6f: validation at HEAD (after timing mode 2 for partitioned timed calls): smoke, the whole GPU suite, stress, the
# driver-shaped (with cpu_baseline) and default bench lines, rocprofv3 stats of both.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6f
rm -rf $O; mkdir -p $O
S=scripts/gpu_step.sh
R=$GRAFT_REPO_ROOT
$S 300 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
grep -q "smoke ok" $O/smoke.log || exit 1
$S 900 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
tail -2 $O/pytest.log; grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
$S 300 $O/stress.log python -u scripts/stress_small.py 60 || exit $?
grep -q "done bad=0" $O/stress.log || exit 1
$S 300 $O/bench_driver.json python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
$S 300 $O/bench_default.json python -u bench.py --no-cpu-baseline || exit $?
$S 200 $O/bench_loop_rccl.json python -u bench.py --rank-mode --loopback --steps 20 --warmup 5 --no-cpu-baseline || exit $?
cd /tmp && export TMPDIR=/tmp && cd $R
$S 200 $O/rocprof_default.log rocprofv3 --kernel-trace --stats -d $O/prof_default -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline || exit $?
$S 200 $O/rocprof_driver.log rocprofv3 --kernel-trace --stats -d $O/prof_driver -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
echo done
