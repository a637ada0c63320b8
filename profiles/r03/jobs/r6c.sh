#!/bin/bash
# r6c: the overlapped schedule with its halo on the compute stream behind the ring kernel
# (LIFE_HALO_ON_COMPUTE=1: no ring -> comm-stream hop before the pack) against the comm-stream halo,
# on the one-GPU rehearsal (RCCL loopback in rank mode, LOCAL loopback, 4 LOCAL shards); parity first;
# a kernel trace of the loopback pass with the option on.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6c
rm -rf $O; mkdir -p $O
S=scripts/gpu_step.sh
R=$GRAFT_REPO_ROOT
LIFE_HALO_ON_COMPUTE=1 $S 500 $O/pytest.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_loopback.py tests/test_gpu_rank.py -k "multi_shard or loopback or rank" -x -q --timeout 250 --timeout-method thread -p no:cacheprovider || exit $?
tail -2 $O/pytest.log; grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
for i in 1 2; do
  for h in 0 1; do
    LIFE_HALO_ON_COMPUTE=$h $S 200 $O/rccl20_h${h}_$i.json python -u bench.py --rank-mode --loopback --steps 20 --warmup 5 --no-cpu-baseline || exit $?
    LIFE_HALO_ON_COMPUTE=$h $S 200 $O/rccl992_h${h}_$i.json python -u bench.py --rank-mode --loopback --no-cpu-baseline || exit $?
    LIFE_HALO_ON_COMPUTE=$h $S 200 $O/local20_h${h}_$i.json python -u bench.py --loopback --steps 20 --warmup 5 --no-cpu-baseline || exit $?
    LIFE_HALO_ON_COMPUTE=$h $S 300 $O/strong4_h${h}_$i.json python -u bench.py --gpus 4 --scaling strong --steps 64 --warmup 32 --no-cpu-baseline || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp && cd $R
LIFE_HALO_ON_COMPUTE=1 $S 200 $O/trace.log rocprofv3 --kernel-trace -d $O/trace_h1 -o run --output-format csv -- python3 $R/bench.py --rank-mode --loopback --steps 20 --warmup 5 --no-cpu-baseline || exit $?
echo done
