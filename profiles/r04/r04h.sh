#!/bin/bash
# r04h: bit tile: this build vs r4b vs 64-B aligned loops (-falign-loops=64);
# byte tile: 2 tiles per CU (this build) vs 3 (LIFE_BYTE_WPE=6 with the load
# phase fenced every 2 / 1 rows, 74 VGPRs, no spills).  Orders alternate.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r04/h; mkdir -p $O
S=scripts/gpu_step.sh
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  if [ "$lib" = cur ]; then $S 150 $O/$n.log python -u bench.py "$@" --no-cpu-baseline || return $?
  else LIFE_MI355X_LIB=$R/build_exp/$lib/liblife_mi355x.so $S 150 $O/$n.log python -u bench.py "$@" --no-cpu-baseline || return $?; fi
}
i=0
for v in cur r4b al64 al64 r4b cur cur al64 r4b; do i=$((i+1)); run bit_${v}_$i $v --steps 20 --warmup 5 || exit $?; done
i=0
for v in cur b6c2 b6c1 b6c1 b6c2 cur; do i=$((i+1)); run byte_${v}_$i $v --kernel byte --steps 64 --warmup 32 || exit $?; done
echo done
