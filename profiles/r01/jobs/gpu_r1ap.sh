#!/bin/bash
# Drifting frame A/B: drift1 (default build) vs drift0 (centred frame) vs drift2 (DPP left), bit + byte, 3 rounds; drift1 row heights.
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1ap; mkdir -p $O
S=$R/scripts/gpu_step.sh
for rnd in 1 2 3; do
  for v in default drift0 drift2; do
    for k in bit byte; do
      if [ $v = default ]; then unset LIFE_MI355X_LIB; else export LIFE_MI355X_LIB=$R/build_exp/$v/liblife_mi355x.so; fi
      $S 120 $O/b.log python -u bench.py --kernel $k --no-cpu-baseline --steps 320
      python3 -c "import json,sys; d=json.loads([l for l in open('$O/b.log') if l.startswith('{')][0]); print(json.dumps({'round':$rnd,'variant':'$v','kernel':'$k','value':d['value'],'kernel_ms':d['roofline']['kernel_avg_ms']}))" | tee -a $O/ab.jsonl
    done
  done
done
unset LIFE_MI355X_LIB
for rows in 40 56; do
  LIFE_TEMPORAL_ROWS=$rows $S 120 $O/b.log python -u bench.py --kernel bit --no-cpu-baseline --steps 320
  python3 -c "import json; d=json.loads([l for l in open('$O/b.log') if l.startswith('{')][0]); print(json.dumps({'variant':'drift1_rows$rows','kernel':'bit','value':d['value'],'kernel_ms':d['roofline']['kernel_avg_ms']}))" | tee -a $O/ab.jsonl
done
