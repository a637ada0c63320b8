#!/bin/bash
set -e
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r1g; mkdir -p $O
R=$GRAFT_REPO_ROOT
S=$R/scripts/gpu_step.sh
$S 600 $O/pytest_gpu.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tail -4 $O/pytest_gpu.log
$S 300 $O/tune_t.log python -u scripts/tune.py --temporal 48,64,80,96 --gens 4
cat $O/tune_t.log
$S 240 $O/bench_bit.log python -u bench.py --kernel bit
grep '^{' $O/bench_bit.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $R/$O/counters_list.txt 2>&1 || true
$S 300 $R/$O/rocprof_bit.log rocprofv3 --kernel-trace --stats -d $R/$O/prof_bit -o run --output-format csv -- python3 $R/bench.py --kernel bit --no-cpu-baseline
$S 120 $R/$O/pmc_fetch.log timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE -d $R/$O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --kernel bit --steps 16 --warmup 8 --no-cpu-baseline
$S 120 $R/$O/pmc_write.log timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE -d $R/$O/pmc_write -o run --output-format csv -- python3 $R/bench.py --kernel bit --steps 16 --warmup 8 --no-cpu-baseline
$S 120 $R/$O/pmc_sq.log timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT -d $R/$O/pmc_sq -o run --output-format csv -- python3 $R/bench.py --kernel bit --steps 16 --warmup 8 --no-cpu-baseline
ls $R/$O
