#!/bin/bash
# A/B: neighbour words by DPP + ds_bpermute (hsum2, default) vs one LDS
# write + ds_read2 (hsum3); parity of hsum3 on the temporal tests first.
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1w; mkdir -p $O
S=$R/scripts/gpu_step.sh
LIFE_MI355X_LIB=$R/build_exp/hsum3/liblife_mi355x.so $S 300 $O/pytest_hsum3.log python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "temporal or small" --timeout 180 --timeout-method thread
tail -2 $O/pytest_hsum3.log
for rnd in 1 2; do
  for v in hsum2 hsum3; do
    for k in bit byte; do
      LIFE_MI355X_LIB=$R/build_exp/$v/liblife_mi355x.so $S 200 $O/bench_${v}_${k}_$rnd.log python -u bench.py --kernel $k --no-cpu-baseline
      echo "$v $k $rnd $(grep '^{' $O/bench_${v}_${k}_$rnd.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["kernel_avg_ms"], d.get("valu",{}).get("frac"))')"
    done
  done
done
