#!/bin/bash
# Round-1 validation of the stacked-wave temporal kernel (K=16, 64 rows/wave): GPU parity suite, smoke,
# bench lines (bit / byte / p46gun_big), rocprofv3 kernel-trace stats and
# separate PMC passes for the dominant kernels.
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1k; mkdir -p $O
S=$R/scripts/gpu_step.sh
$S 600 $O/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
tail -3 $O/pytest_gpu.log
$S 120 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()"
tail -1 $O/smoke.log
$S 240 $O/bench_bit.log python -u bench.py
grep '^{' $O/bench_bit.log | cut -c1-300
$S 240 $O/bench_byte.log python -u bench.py --kernel byte --steps 30 --no-cpu-baseline
grep '^{' $O/bench_byte.log | cut -c1-300
$S 240 $O/bench_p46.log python -u bench.py --workload p46gun_big --steps 10000 --warmup 10 --no-cpu-baseline
grep '^{' $O/bench_p46.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
$S 300 $O/rocprof_bit.log rocprofv3 --kernel-trace --stats -d $O/prof_bit -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline
$S 300 $O/rocprof_byte.log rocprofv3 --kernel-trace --stats -d $O/prof_byte -o run --output-format csv -- python3 $R/bench.py --kernel byte --steps 30 --no-cpu-baseline
$S 120 $O/pmc_fetch_bit.log timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_bit -o run --output-format csv -- python3 $R/bench.py --steps 16 --warmup 8 --no-cpu-baseline
$S 120 $O/pmc_write_bit.log timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_bit -o run --output-format csv -- python3 $R/bench.py --steps 16 --warmup 8 --no-cpu-baseline
$S 120 $O/pmc_sq_bit.log timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT -d $O/pmc_sq_bit -o run --output-format csv -- python3 $R/bench.py --steps 16 --warmup 8 --no-cpu-baseline
$S 120 $O/pmc_fetch_byte.log timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch_byte -o run --output-format csv -- python3 $R/bench.py --kernel byte --steps 5 --warmup 1 --no-cpu-baseline
$S 120 $O/pmc_write_byte.log timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write_byte -o run --output-format csv -- python3 $R/bench.py --kernel byte --steps 5 --warmup 1 --no-cpu-baseline
find $O -name '*.csv' | sort
