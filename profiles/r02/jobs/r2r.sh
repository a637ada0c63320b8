#!/bin/bash
# r2r: flow default: full GPU suite, smoke, bench lines, rocprofv3 stats + PMC of the default bench, frames at scale
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2r
mkdir -p $O
S=scripts/gpu_step.sh
R=$GRAFT_REPO_ROOT
$S 1200 $O/pytest.log python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread || exit $?
grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
$S 300 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
$S 300 $O/bench_default.json python -u bench.py || exit $?
$S 300 $O/bench_byte.json python -u bench.py --kernel byte --no-cpu-baseline || exit $?
$S 300 $O/bench_32768.json python -u bench.py --size 32768 --no-cpu-baseline || exit $?
$S 300 $O/bench_32768_byte.json python -u bench.py --size 32768 --kernel byte --no-cpu-baseline || exit $?
$S 300 $O/bench_driver.json python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
$S 300 $O/bench_p46.json python -u bench.py --workload p46gun_big --steps 10000 --warmup 16 --no-cpu-baseline || exit $?
$S 300 $O/rocprof_bit.log rocprofv3 --kernel-trace --stats -d $O/prof_bit -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  $S 120 $O/pmc_$c.log timeout -s KILL 100 rocprofv3 --pmc $c -d $O/pmc_$c -o run --output-format csv -- python3 $R/bench.py --steps 80 --warmup 40 --no-cpu-baseline || exit $?
done
$S 120 $O/pmc_SQ.log timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $O/pmc_SQ -o run --output-format csv -- python3 $R/bench.py --steps 80 --warmup 40 --no-cpu-baseline || exit $?
df -h /dev/shm /tmp > $O/df.txt 2>&1
$S 600 $O/frames.json python -u scripts/frames_at_scale.py --n 32768 --gens 1000 --save 100 --dir /dev/shm || exit $?
for round in 1 2; do
  for size in 65536 32768; do
    $S 300 $O/byte_flow_${size}_$round.json env LIFE_FLOW_BYTE=1 python -u bench.py --kernel byte --size $size --no-cpu-baseline --steps 480 --warmup 32 || exit $?
    $S 300 $O/byte_tiles_${size}_$round.json env LIFE_FLOW_BYTE=0 python -u bench.py --kernel byte --size $size --no-cpu-baseline --steps 480 --warmup 32 || exit $?
  done
done
