#!/bin/bash
# r5m: serial schedule for partitioned temporal shards (LIFE_OPT_OVERLAP 0: all tiles in one launch,
# then the halo) vs the overlapped ring / interior / halo schedule, on the one-GPU rehearsal of the
# multi-GPU path (loopback over RCCL in rank mode, and over LOCAL copies).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5m
mkdir -p $O
S=scripts/gpu_step.sh
$S 500 $O/pytest.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_loopback.py -k "multi_shard or loopback" -x -q --timeout 250 --timeout-method thread -p no:cacheprovider || exit $?
tail -2 $O/pytest.log; grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
for i in 1 2; do
  for ov in "" "--no-overlap"; do
    t=${ov:+serial}; t=${t:-overlap}
    $S 200 $O/rccl20_${t}_$i.json python -u bench.py --rank-mode --loopback --steps 20 --warmup 5 --no-cpu-baseline $ov || exit $?
    $S 200 $O/rccl992_${t}_$i.json python -u bench.py --rank-mode --loopback --no-cpu-baseline $ov || exit $?
    $S 200 $O/local20_${t}_$i.json python -u bench.py --loopback --steps 20 --warmup 5 --no-cpu-baseline $ov || exit $?
  done
done
echo done
