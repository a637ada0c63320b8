#!/bin/bash
# r3i: PMC passes of the byte tiles at HEAD (R = 48, K = 32): HBM bytes per launch for profiles/traffic.json
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3i
mkdir -p $O
S=scripts/gpu_step.sh
R=$GRAFT_REPO_ROOT
for c in FETCH_SIZE WRITE_SIZE; do
  $S 120 $O/pmc_$c.log timeout -s KILL 100 rocprofv3 --pmc $c -d $O/pmc_$c -o run --output-format csv -- python3 $R/bench.py --kernel byte --steps 64 --warmup 32 --no-cpu-baseline || exit $?
done
$S 120 $O/pmc_SQ.log timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $O/pmc_SQ -o run --output-format csv -- python3 $R/bench.py --kernel byte --steps 64 --warmup 32 --no-cpu-baseline || exit $?
$S 200 $O/rocprof_byte.log rocprofv3 --kernel-trace --stats -d $O/prof_byte -o run --output-format csv -- python3 $R/bench.py --kernel byte --no-cpu-baseline || exit $?
