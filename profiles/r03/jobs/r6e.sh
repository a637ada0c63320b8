#!/bin/bash
# r6e: r6c's halo-on-compute-stream schedule (LIFE_HALO_ON_COMPUTE=1) re-measured now that the timed
# call carries no phase events (r6d): parity, then A/B on the loopback rehearsals.  (Mixed: RCCL 20
# generations equal, 992 +2 %, LOCAL 20 -2..-6 %; not kept, the knob was removed after this job.)
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6e
rm -rf $O; mkdir -p $O
S=scripts/gpu_step.sh
LIFE_HALO_ON_COMPUTE=1 $S 500 $O/pytest.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_loopback.py tests/test_gpu_rank.py -k "multi_shard or loopback or rank" -x -q --timeout 250 --timeout-method thread -p no:cacheprovider || exit $?
tail -2 $O/pytest.log; grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
for i in 1 2; do
  for h in 0 1; do
    LIFE_HALO_ON_COMPUTE=$h $S 200 $O/rccl20_h${h}_$i.json python -u bench.py --rank-mode --loopback --steps 20 --warmup 5 --no-cpu-baseline || exit $?
    LIFE_HALO_ON_COMPUTE=$h $S 200 $O/rccl992_h${h}_$i.json python -u bench.py --rank-mode --loopback --no-cpu-baseline || exit $?
    LIFE_HALO_ON_COMPUTE=$h $S 200 $O/local20_h${h}_$i.json python -u bench.py --loopback --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  done
done
echo done
