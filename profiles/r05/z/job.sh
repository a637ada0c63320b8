#!/bin/bash
# r05z: HBM traffic of configs[2] (32768^2) for its bench line's
# roofline.traffic: FETCH_SIZE / WRITE_SIZE passes of the dataflow call (one
# launch of 8 x 12 generations) and of the byte tiles (2 launches of 32).
# Expectation: dataflow ~1.05-1.2x the compulsory 0.0625 GB per pass (sc1
# window loads, per-item order without XCD runs); byte ~1.13x as at 65536^2.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r05/z; mkdir -p $O
S=scripts/gpu_step.sh
cd /tmp && export TMPDIR=/tmp && cd $R
for c in FETCH_SIZE WRITE_SIZE; do
  $S 90 $O/pmc_${c}_flow.log timeout -s KILL 80 rocprofv3 --pmc $c -d $O/pmc_${c}_flow -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --shape 32768x32768 --steps 96 --warmup 32 || exit $?
  $S 90 $O/pmc_${c}_byte.log timeout -s KILL 80 rocprofv3 --pmc $c -d $O/pmc_${c}_byte -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --shape 32768x32768 --kernel byte --steps 64 --warmup 32 || exit $?
done
echo done
