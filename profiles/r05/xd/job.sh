#!/bin/bash
# r05xd: an exchange-block interior of more than one round of workgroups as
# two launches in its stream -- its first ~round (slots - 16), then the rest.
# r05xc: a one-workgroup-per-tile interior refills every slot until its last
# tile is dispatched, so the RCCL kernel queued behind the ring starts only
# then; between two launches the slots the first frees can go to it.
# Expectation: the halo beside a 65536^2 interior 0.33 -> ~0.05-0.1 ms, the
# block 0.445 -> ~0.42 ms (+2-4 % on the 20-generation loopback line and the
# 8-GPU weak lines); small shards unchanged (their interiors fit one round).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/xd; mkdir -p $O
S=scripts/gpu_step.sh
$S 900 $O/test_part.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_loopback.py tests/test_gpu_poison.py -k "deep_halo or loopback or multi_shard or temporal_multi" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/test_part.log && ! grep -q -E "[0-9]+ (failed|error)" $O/test_part.log || exit 1
for i in 1 2; do
  for r in 0 16 64; do
    LIFE_INTERIOR_SPLIT=$r $S 150 $O/loop20_r${r}_$i.log python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 20 --warmup 5 || exit $?
  done
done
L="python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 96 --warmup 32"
for sh in 32768x65536 65536x65536; do
  for r in 0 16; do
    LIFE_INTERIOR_SPLIT=$r $S 150 $O/loop_${sh}_r$r.log $L --shape $sh || exit $?
  done
done
for r in 0 16; do
  LIFE_INTERIOR_SPLIT=$r $S 300 $O/weak8_r$r.log python -u bench.py --gpus 8 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
$S 150 $O/trace_loop20.log timeout -s KILL 140 rocprofv3 --kernel-trace -d $O/trace_loop20 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 20 --warmup 5 || exit $?
echo done
