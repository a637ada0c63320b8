#!/bin/bash
# r04i: VGPR-bank A/B of the bit tile: this build (LIFE_BIT_PAD=1, 10
# three-source-one-bank ops per generation) vs pad0 (155) vs r4b (11), ABC
# orders alternating; parity subset of the store-lane rewrite.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r04/i; mkdir -p $O
S=scripts/gpu_step.sh
$S 600 $O/parity.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "deep_halo or temporal or wide_periodic or band" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/parity.log && ! grep -q -E "[0-9]+ (failed|error)" $O/parity.log || exit 1
run() {  # name lib args...
  local n=$1 lib=$2; shift 2
  if [ "$lib" = cur ]; then $S 150 $O/$n.log python -u bench.py "$@" --no-cpu-baseline || return $?
  else LIFE_MI355X_LIB=$R/build_exp/$lib/liblife_mi355x.so $S 150 $O/$n.log python -u bench.py "$@" --no-cpu-baseline || return $?; fi
}
i=0
for v in cur pad0 r4b r4b pad0 cur cur pad0 r4b; do i=$((i+1)); run bit_${v}_$i $v --steps 20 --warmup 5 || exit $?; done
i=0
for v in cur pad0 pad0 cur; do i=$((i+1)); run loop_${v}_$i $v --steps 20 --warmup 5 --rank-mode --loopback --no-parity || exit $?; done
echo done
