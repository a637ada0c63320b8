#!/bin/bash
# r04d: diagnose the weak-2 parity failure (deep halo vs peer-only LOCAL order)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04/d; mkdir -p $O
S=scripts/gpu_step.sh
$S 300 $O/deep_tests.log python -u -m pytest tests/test_gpu_parity.py -k "deep_halo or temporal_multi_shard" -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
for dh in 0 1; do
  LIFE_DEEP_HALO=$dh $S 120 $O/w2_d$dh.log python -u bench.py --gpus 2 --size 8192 --steps 45 --warmup 4 --no-cpu-baseline || exit $?
done
LIFE_DEEP_HALO=1 $S 120 $O/w2_d1_serial.log python -u bench.py --gpus 2 --size 8192 --steps 45 --warmup 4 --no-overlap --no-cpu-baseline || exit $?
echo done
