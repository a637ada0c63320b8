#!/bin/bash
# r05xc: the exchange block's interior as a persistent launch that leaves 8
# resident slots free (LIFE_PERSIST_RESERVE, tstep_bit_persist_kernel).
# r05w / xb: the RCCL kernel, queued behind the ring while the interior's
# one-workgroup-per-tile launch holds every slot, ended within 5 us of the
# interior (14 us alone) whatever the stream priority -- no slot an RCCL
# workgroup fits into frees up until the interior's last tiles are
# dispatched.  Expectation: the halo beside a 65536^2 interior drops from
# ~0.33 ms to ~0.05 ms, the block to about the interior (0.45 -> ~0.42 ms):
# the 20-generation loopback line +3-5 % (94 -> ~98 T), the 8-GPU weak
# lines the same.  Parity of every partitioned path first.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/xc; mkdir -p $O
S=scripts/gpu_step.sh
$S 900 $O/test_part.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_loopback.py tests/test_gpu_poison.py -k "deep_halo or loopback or multi_shard or temporal_multi" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/test_part.log && ! grep -q -E "[0-9]+ (failed|error)" $O/test_part.log || exit 1
for i in 1 2; do
  for r in 0 8; do
    LIFE_PERSIST_RESERVE=$r $S 150 $O/loop20_r${r}_$i.log python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 20 --warmup 5 || exit $?
  done
done
L="python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 96 --warmup 32"
for sh in 16384x32768 32768x32768 65536x65536; do
  for r in 0 8 16; do
    LIFE_PERSIST_RESERVE=$r $S 150 $O/loop_${sh}_r$r.log $L --shape $sh || exit $?
  done
done
for r in 0 8; do
  LIFE_PERSIST_RESERVE=$r $S 300 $O/weak8_r$r.log python -u bench.py --gpus 8 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
$S 150 $O/trace_loop20.log timeout -s KILL 140 rocprofv3 --kernel-trace -d $O/trace_loop20 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 20 --warmup 5 || exit $?
echo done
