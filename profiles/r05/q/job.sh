#!/bin/bash
# r05q: thin ring x CU-masked interior.  r05p: the thin ring cut the ring
# 38 -> 27 us (16384x32768) and 87 -> 35 us (65536^2), but the RCCL kernel
# then ran 18 -> 40 us beside the interior tiles (3 tile workgroups per CU
# around its 4), so the block did not shrink.  LIFE_COMM_CUS=1 runs the
# interior on a stream whose CU mask leaves one CU of every 32 free for the
# halo kernels.  Expectation: with both, the 16384x32768 block ~0.107 ->
# ~0.08 ms (+8-10 % on the line); 65536^2 flat to +2 %.  Parity of the
# masked schedule first.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/q; mkdir -p $O
S=scripts/gpu_step.sh
LIFE_COMM_CUS=1 $S 600 $O/test_cus.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_loopback.py -k "thin_ring or deep_halo or loopback" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/test_cus.log && ! grep -q -E "[0-9]+ (failed|error)" $O/test_cus.log || exit 1
L="python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 96 --warmup 32"
for i in 1 2; do
  for t in 0 1; do
    for c in 0 1; do
      LIFE_THIN_RING=$t LIFE_COMM_CUS=$c $S 150 $O/loop_16384x32768_r${t}c${c}_$i.log $L --shape 16384x32768 || exit $?
    done
  done
done
for sh in 32768x32768 65536x65536; do
  for t in 0 1; do
    for c in 0 1; do
      LIFE_THIN_RING=$t LIFE_COMM_CUS=$c $S 150 $O/loop_${sh}_r${t}c$c.log $L --shape $sh || exit $?
    done
  done
done
for t in 0 1; do
  for c in 0 1; do
    LIFE_THIN_RING=$t LIFE_COMM_CUS=$c $S 300 $O/weak8_r${t}c$c.log python -u bench.py --gpus 8 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
LIFE_COMM_CUS=1 $S 150 $O/trace_loop.log timeout -s KILL 140 rocprofv3 --kernel-trace -d $O/trace_loop -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 96 --warmup 32 --shape 16384x32768 || exit $?
echo done
