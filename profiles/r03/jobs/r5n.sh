#!/bin/bash
# r5n: bit one-generation rows x depth sweep with and without the XCD strip order.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5n
mkdir -p $O
S=scripts/gpu_step.sh
for x in 1 0; do
  LIFE_XCD_ORDER_ONEGEN=$x LIFE_TEMPORAL_DEPTH=1 $S 300 $O/tune_bit1_x$x.log python -u scripts/tune.py --kernels bit --rows 16,32,64 --depths 2,4,8,18 --gens 10 --rounds 3 || exit $?
done
echo done
