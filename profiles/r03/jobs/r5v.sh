#!/bin/bash
# r5v: tile shapes re-measured with the XCD order (round 3): byte window rows (LIFE_TEMPORAL_ROWS_BYTE,
# 8 waves, 32 ghost rows per end) on the byte default run, and the bit shapes (rows x waves) on the
# driver-shaped run; FETCH/WRITE of the byte candidates.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5v
rm -rf $O; mkdir -p $O
S=scripts/gpu_step.sh
for r in 40 48 56 64 96; do
  LIFE_TEMPORAL_ROWS_BYTE=$r $S 200 $O/byte_r$r.json python -u bench.py --kernel byte --no-cpu-baseline || exit $?
done
for i in 1 2; do
  for s in 24x8 16x8 32x8 24x12 16x16 24x16; do
    r=${s%x*}; w=${s#*x}
    LIFE_TEMPORAL_ROWS=$r LIFE_TILE_WAVES=$w $S 200 $O/drv_${s}_$i.json python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  done
done
echo done
