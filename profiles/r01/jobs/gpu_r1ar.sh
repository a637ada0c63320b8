#!/bin/bash
# Bench warm-up study: kernel time falls over the first launches (clock ramp); value vs warmup/steps.
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1ar; mkdir -p $O
S=$R/scripts/gpu_step.sh
for ws in "32 160" "320 640" "960 960" "3200 3200" "32 160"; do
  set -- $ws
  $S 120 $O/b.log python -u bench.py --no-cpu-baseline --warmup $1 --steps $2
  python3 -c "import json; d=json.loads([l for l in open('$O/b.log') if l.startswith('{')][0]); print(json.dumps({'warmup':$1,'steps':$2,'value':d['value'],'kernel_ms':d['roofline']['kernel_avg_ms'],'launches':d['roofline']['kernel_launches']}))" | tee -a $O/warmup.jsonl
done
