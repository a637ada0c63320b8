#!/bin/bash
# r2t: dataflow pass size sweep (LIFE_BLOCK_GENS) incl. the driver's 20-generation call; PMC passes of the default bench; frames at scale; reference mpirun cpu_baseline on the box
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2t
mkdir -p $O
S=scripts/gpu_step.sh
R=$GRAFT_REPO_ROOT
for m in 8 10 12 16 20; do
  $S 200 $O/flow_m${m}_65536.json env LIFE_BLOCK_GENS=$m python -u bench.py --no-cpu-baseline --steps 480 --warmup 48 || exit $?
  $S 200 $O/flow_m${m}_32768.json env LIFE_BLOCK_GENS=$m python -u bench.py --no-cpu-baseline --size 32768 --steps 480 --warmup 48 || exit $?
  $S 200 $O/driver_m${m}.json env LIFE_BLOCK_GENS=$m python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 || exit $?
done
$S 300 $O/bench_default_cpu.json python -u bench.py || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  $S 120 $O/pmc_$c.log timeout -s KILL 100 rocprofv3 --pmc $c -d $O/pmc_$c -o run --output-format csv -- python3 $R/bench.py --steps 80 --warmup 40 --no-cpu-baseline || exit $?
done
$S 120 $O/pmc_SQ.log timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $O/pmc_SQ -o run --output-format csv -- python3 $R/bench.py --steps 80 --warmup 40 --no-cpu-baseline || exit $?
$S 600 $O/frames.json python -u scripts/frames_at_scale.py --n 32768 --gens 1000 --save 100 --dir /dev/shm || exit $?
