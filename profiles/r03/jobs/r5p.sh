#!/bin/bash
# r5p: validation at HEAD: smoke, the whole GPU suite, stress; the bench lines (driver shape with
# cpu_baseline, default, byte, 32768^2, p46gun_big, byte / bit one-generation, RCCL loopback, 4 LOCAL
# shards); rocprofv3 stats + trace of the driver-shaped and default runs; PMC traffic + SQ of the
# driver-shaped launch.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5p
mkdir -p $O
S=scripts/gpu_step.sh
R=$GRAFT_REPO_ROOT
$S 300 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
grep -q "smoke ok" $O/smoke.log || exit 1
$S 900 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
tail -2 $O/pytest.log; grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
$S 300 $O/stress.log python -u scripts/stress_small.py 40 || exit $?
grep -q "done bad=0" $O/stress.log || exit 1
$S 300 $O/bench_driver.json python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
$S 300 $O/bench_default.json python -u bench.py --no-cpu-baseline || exit $?
$S 200 $O/bench_byte.json python -u bench.py --kernel byte --no-cpu-baseline || exit $?
$S 200 $O/bench_32768.json python -u bench.py --size 32768 --no-cpu-baseline || exit $?
$S 200 $O/bench_p46.json python -u bench.py --workload p46gun_big --steps 10000 --warmup 16 --no-cpu-baseline || exit $?
LIFE_TEMPORAL_DEPTH_BYTE=1 $S 200 $O/bench_byte1.json python -u bench.py --kernel byte --steps 30 --warmup 10 --no-cpu-baseline || exit $?
LIFE_TEMPORAL_DEPTH=1 $S 200 $O/bench_bit1.json python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline || exit $?
$S 200 $O/bench_loop_rccl.json python -u bench.py --rank-mode --loopback --steps 20 --warmup 5 --no-cpu-baseline || exit $?
$S 300 $O/bench_strong4.json python -u bench.py --gpus 4 --scaling strong --steps 64 --warmup 32 --no-cpu-baseline || exit $?
cd /tmp && export TMPDIR=/tmp && cd $R
$S 200 $O/rocprof_default.log rocprofv3 --kernel-trace --stats -d $O/prof_default -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline || exit $?
$S 200 $O/rocprof_driver.log rocprofv3 --kernel-trace --stats -d $O/prof_driver -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  $S 120 $O/pmc_$c.log timeout -s KILL 100 rocprofv3 --pmc $c -d $O/pmc_$c -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
done
$S 120 $O/pmc_SQ.log timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $O/pmc_SQ -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
echo done
