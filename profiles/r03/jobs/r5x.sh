#!/bin/bash
# r5x: the driver-shaped call (20 generations) as ONE launch of m = 20 (LIFE_BLOCK_GENS=20) against
# the default two launches of 10, on the 24x8 tile and the taller 24x12 / 16x16 windows.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5x
rm -rf $O; mkdir -p $O
S=scripts/gpu_step.sh
for i in 1 2; do
  $S 200 $O/drv_base_$i.json python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  for s in 24x8 24x12 16x16; do
    r=${s%x*}; w=${s#*x}
    LIFE_BLOCK_GENS=20 LIFE_TEMPORAL_ROWS=$r LIFE_TILE_WAVES=$w $S 200 $O/drv_m20_${s}_$i.json python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  done
  LIFE_BLOCK_GENS=20 LIFE_TEMPORAL_ROWS=24 LIFE_TILE_WAVES=12 $S 200 $O/def_m20_24x12_$i.json python -u bench.py --no-cpu-baseline || exit $?
done
echo done
