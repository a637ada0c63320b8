#!/bin/bash
# r5y: do the bit tiles' load / compute / store phases run in lock-step across the chip?  First-round
# workgroups staggered by sleeps (LIFE_STAGGER = 4-us sleeps per level, 3 levels) or every workgroup
# given a wave priority by level (LIFE_PRIO), level from the dispatch index (LIFE_STAGGER_MODE),
# on the driver-shaped call.  (No gain -- sleeps 98.1-102.5, priorities 94.8-96.2 against 102.5-103.4 T;
# the knobs were removed after this job)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5y
rm -rf $O; mkdir -p $O
S=scripts/gpu_step.sh
for i in 1 2; do
  $S 200 $O/drv_base_$i.json python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  for v in "2 0 0" "4 0 0" "4 1 0" "4 2 0" "0 0 1" "0 1 1" "0 2 1"; do
    set -- $v
    LIFE_STAGGER=$1 LIFE_STAGGER_MODE=$2 LIFE_PRIO=$3 $S 200 $O/drv_s$1_m$2_p$3_$i.json python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  done
done
echo done
