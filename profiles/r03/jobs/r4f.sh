#!/bin/bash
# r4f: timing modes (call pair / per-launch record / dispatch-stamped / off) on the driver shape,
# and the per-generation cost against passes per call, tiles vs dataflow (flow forced from 2 passes)
O=gpurun_out/r4f; mkdir -p $O
for mode in 0 1 2 3; do for i in 1 2 3; do
  LIFE_TIMING_MODE=$mode timeout -k 10 120 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/drv_mode${mode}_$i.json 2>> $O/err.log || exit 1
done; done
LIFE_FLOW_MIN_PASSES=2 timeout -k 10 300 python scripts/pass_study.py $O/pass_study.jsonl
