#!/bin/bash
# r4g: dataflow vs per-launch tiles on the long default run (992 generations), pass sizes 10-16, alternated
O=gpurun_out/r4g; mkdir -p $O
for rep in 1 2; do for m in 10 12 14 16; do for flow in 0 1; do
  LIFE_BLOCK_GENS=$m timeout -k 10 120 python bench.py --no-cpu-baseline --flow $flow > $O/def_m${m}_f${flow}_$rep.json 2>> $O/err.log || exit 1
  python3 -c "import json; d=json.load(open('$O/def_m${m}_f${flow}_$rep.json')); r=d['roofline']; print($m, $flow, d['value'], r['kernel_avg_ms'], d['config']['kernel_path'])"
done; done; done
