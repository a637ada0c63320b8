#!/bin/bash
# Final round-1 measurement set: parity suite, smoke, bench lines, rocprof
# kernel-trace stats and separate PMC passes for both temporal kernels.
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1s; mkdir -p $O
S=$R/scripts/gpu_step.sh
$S 500 $O/pytest_gpu.log python -u -m pytest tests -m gpu -q --timeout 180 --timeout-method thread
tail -2 $O/pytest_gpu.log
$S 120 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
tail -1 $O/smoke.log
$S 240 $O/bench_bit.log python -u bench.py
grep '^{' $O/bench_bit.log | cut -c1-200
$S 240 $O/bench_byte.log python -u bench.py --kernel byte --no-cpu-baseline
grep '^{' $O/bench_byte.log | cut -c1-200
$S 240 $O/bench_p46.log python -u bench.py --workload p46gun_big --steps 10000 --warmup 16 --no-cpu-baseline
grep '^{' $O/bench_p46.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
$S 300 $O/rocprof_bit.log rocprofv3 --kernel-trace --stats -d $O/prof_bit -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline
$S 300 $O/rocprof_byte.log rocprofv3 --kernel-trace --stats -d $O/prof_byte -o run --output-format csv -- python3 $R/bench.py --kernel byte --no-cpu-baseline
for k in bit byte; do
  $S 120 $O/pmc_fetch_$k.log timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_$k -o run --output-format csv -- python3 $R/bench.py --kernel $k --steps 64 --warmup 32 --no-cpu-baseline
  $S 120 $O/pmc_write_$k.log timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_$k -o run --output-format csv -- python3 $R/bench.py --kernel $k --steps 64 --warmup 32 --no-cpu-baseline
  $S 120 $O/pmc_sq_$k.log timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT -d $O/pmc_sq_$k -o run --output-format csv -- python3 $R/bench.py --kernel $k --steps 64 --warmup 32 --no-cpu-baseline
done
ls $O
