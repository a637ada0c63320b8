#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r1d; mkdir -p $O
R=$GRAFT_REPO_ROOT
S=$R/scripts/gpu_step.sh
$S 240 $O/bench_bit.log python -u bench.py --kernel bit
tail -1 $O/bench_bit.log
$S 240 $O/bench_byte.log python -u bench.py --kernel byte --steps 30 --no-cpu-baseline
tail -1 $O/bench_byte.log
$S 240 $O/bench_p46.log python -u bench.py --workload p46gun_big --steps 10000 --warmup 10 --no-cpu-baseline
tail -1 $O/bench_p46.log
cd /tmp && export TMPDIR=/tmp
$S 300 $R/$O/rocprof_bit.log rocprofv3 --kernel-trace --stats -d $R/$O/prof_bit -o run --output-format csv -- python3 $R/bench.py --kernel bit --no-cpu-baseline
$S 300 $R/$O/rocprof_byte.log rocprofv3 --kernel-trace --stats -d $R/$O/prof_byte -o run --output-format csv -- python3 $R/bench.py --kernel byte --steps 30 --no-cpu-baseline
for k in bit byte; do
  $S 120 $R/$O/pmc_fetch_$k.log timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE -d $R/$O/pmc_fetch_$k -o run --output-format csv -- python3 $R/bench.py --kernel $k --steps 5 --warmup 1 --no-cpu-baseline
  $S 120 $R/$O/pmc_write_$k.log timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE -d $R/$O/pmc_write_$k -o run --output-format csv -- python3 $R/bench.py --kernel $k --steps 5 --warmup 1 --no-cpu-baseline
done
find $R/$O -name '*.csv' | head -40
