#!/bin/bash
# r05n: the tail split chosen by a list-scheduling model of the launch
# (LIFE_TAIL_SPLIT 2, scripts/tail_model.py) against the round-4 rule (1).
# Expectation: the driver-shaped 65536^2 call (two launches of 10
# generations, 6494 tiles on 768 slots) drops from 9.0 to 8.5 tile-times in
# the model: up to 5 % off the kernel time, if half tiles really cost half.
# Parity of the split paths first; ABAB pairs of the driver line.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/n; mkdir -p $O
S=scripts/gpu_step.sh
$S 400 $O/test_split.log python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -k "tail_split or driver_shape or temporal_single_shard or deep_halo" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/test_split.log && ! grep -q -E "[0-9]+ (failed|error)" $O/test_split.log || exit 1
for i in 1 2 3; do
  for t in 1 2; do
    LIFE_TAIL_SPLIT=$t $S 120 $O/drv_t${t}_$i.log python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  done
done
for t in 1 2; do
  LIFE_TAIL_SPLIT=$t $S 120 $O/def_t$t.log python -u bench.py --no-cpu-baseline || exit $?
  LIFE_TAIL_SPLIT=$t $S 150 $O/loop_t$t.log python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 96 --warmup 32 --shape 16384x32768 || exit $?
  LIFE_TAIL_SPLIT=$t $S 120 $O/tiles32k_t$t.log python -u bench.py --no-cpu-baseline --shape 32768x32768 --flow 0 || exit $?
done
echo done
