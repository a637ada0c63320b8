#!/bin/bash
# r3j: why the byte dataflow form is slow: PMC bytes and SQ counters of the byte flow vs byte tiles (same call)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3j
mkdir -p $O
S=scripts/gpu_step.sh
R=$GRAFT_REPO_ROOT
for v in flow tiles; do
  case $v in flow) F=1;; tiles) F=0;; esac
  for c in FETCH_SIZE WRITE_SIZE; do
    $S 120 $O/pmc_${c}_$v.log timeout -s KILL 100 env LIFE_FLOW_BYTE=$F rocprofv3 --pmc $c -d $O/pmc_${c}_$v -o run --output-format csv -- python3 $R/bench.py --kernel byte --steps 128 --warmup 32 --no-cpu-baseline || exit $?
  done
  $S 120 $O/pmc_SQ_$v.log timeout -s KILL 100 env LIFE_FLOW_BYTE=$F rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAIT_INST_ANY SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc_SQ_$v -o run --output-format csv -- python3 $R/bench.py --kernel byte --steps 128 --warmup 32 --no-cpu-baseline || exit $?
  $S 120 $O/bench_$v.json env LIFE_FLOW_BYTE=$F python -u bench.py --kernel byte --steps 128 --warmup 32 --no-cpu-baseline || exit $?
done
