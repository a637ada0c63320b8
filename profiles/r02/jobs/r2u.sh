#!/bin/bash
# r2u: driver-shaped 20-generation calls (hot vs cooled soup, loopback LOCAL/RCCL = the per-GPU cost of an N>1 rank),
# byte dataflow A/B, PMC passes of the default bench, frames at scale
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2u
mkdir -p $O
S=scripts/gpu_step.sh
R=$GRAFT_REPO_ROOT
$S 200 $O/driver_w5.json python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 || exit $?
$S 200 $O/driver_w500.json python -u bench.py --no-cpu-baseline --steps 20 --warmup 500 || exit $?
$S 200 $O/driver_loop_local.json python -u bench.py --no-cpu-baseline --steps 20 --warmup 5 --loopback || exit $?
$S 200 $O/driver_loop_rccl.json python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --rank-mode --loopback --steps 20 --warmup 5 --no-cpu-baseline || exit $?
for round in 1 2; do
  for size in 65536 32768; do
    $S 200 $O/byte_flow_${size}_$round.json env LIFE_FLOW_BYTE=1 python -u bench.py --kernel byte --size $size --no-cpu-baseline --steps 480 --warmup 32 || exit $?
    $S 200 $O/byte_tiles_${size}_$round.json env LIFE_FLOW_BYTE=0 python -u bench.py --kernel byte --size $size --no-cpu-baseline --steps 480 --warmup 32 || exit $?
  done
done
for c in FETCH_SIZE WRITE_SIZE; do
  $S 120 $O/pmc_$c.log timeout -s KILL 100 rocprofv3 --pmc $c -d $O/pmc_$c -o run --output-format csv -- python3 $R/bench.py --steps 80 --warmup 40 --no-cpu-baseline || exit $?
done
$S 120 $O/pmc_SQ.log timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d $O/pmc_SQ -o run --output-format csv -- python3 $R/bench.py --steps 80 --warmup 40 --no-cpu-baseline || exit $?
$S 600 $O/frames.json python -u scripts/frames_at_scale.py --n 32768 --gens 1000 --save 100 --dir /dev/shm || exit $?
