#!/bin/bash
# r5c (part B): measurements at the working tree (XCD order for bit + byte tiles, bit one-generation depth 18):
# one-generation XCD order A/B, step(1) calls with one-ghost byte tiles A/B, the bench lines, rocprofv3 stats and
# trace of the default and driver-shaped runs, PMC traffic + SQ of the driver-shaped launch.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${RUN:-r5c}
mkdir -p $O
S=scripts/gpu_step.sh
R=$GRAFT_REPO_ROOT
$S 400 $O/pytest_parity.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_loopback.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider || exit $?
tail -2 $O/pytest_parity.log; grep -q " passed" $O/pytest_parity.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest_parity.log || exit 1
for i in 1 2; do
  for x in 0 1; do
    LIFE_XCD_ORDER_ONEGEN=$x LIFE_TEMPORAL_DEPTH_BYTE=1 $S 200 $O/byte1_x${x}_$i.json python -u bench.py --kernel byte --steps 30 --warmup 10 --no-cpu-baseline || exit $?
    LIFE_XCD_ORDER_ONEGEN=$x LIFE_TEMPORAL_DEPTH=1 $S 200 $O/bit1_x${x}_$i.json python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline || exit $?
  done
done
for i in 1 2; do
  for g in 0 1; do
    LIFE_BYTE_ONE_GHOST=$g $S 200 $O/step1_g${g}_$i.log python -u scripts/step1_rate.py || exit $?
  done
done
$S 300 $O/bench_driver.json python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
$S 300 $O/bench_default.json python -u bench.py --no-cpu-baseline || exit $?
$S 200 $O/bench_byte.json python -u bench.py --kernel byte --no-cpu-baseline || exit $?
$S 200 $O/bench_32768.json python -u bench.py --size 32768 --no-cpu-baseline || exit $?
$S 200 $O/bench_32768_flow.json python -u bench.py --size 32768 --flow 1 --no-cpu-baseline || exit $?
$S 200 $O/bench_p46.json python -u bench.py --workload p46gun_big --steps 10000 --warmup 16 --no-cpu-baseline || exit $?
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
