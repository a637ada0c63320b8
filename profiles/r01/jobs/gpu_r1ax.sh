#!/bin/bash
# Tile height vs grid size (tail rounds): bit and byte at 32768^2 and 65536^2 for several R.
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1ax; mkdir -p $O
S=$R/scripts/gpu_step.sh
for size in 32768 65536; do
  for rows in 32 40 48 56 64; do
    for k in bit byte; do
      if [ $k = bit ]; then export LIFE_TEMPORAL_ROWS=$rows; unset LIFE_TEMPORAL_ROWS_BYTE; else export LIFE_TEMPORAL_ROWS_BYTE=$rows; unset LIFE_TEMPORAL_ROWS; fi
      $S 120 $O/b.log python -u bench.py --size $size --kernel $k --no-cpu-baseline
      python3 -c "import json; d=json.loads([l for l in open('$O/b.log') if l.startswith('{')][0]); print(json.dumps({'size':$size,'kernel':'$k','rows':$rows,'value':d['value'],'kernel_ms':d['roofline']['kernel_avg_ms']}))" | tee -a $O/rows.jsonl
    done
  done
done
