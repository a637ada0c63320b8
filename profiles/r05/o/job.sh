#!/bin/bash
# r05o: trailing halo (LIFE_OPT_TRAIL_HALO 1): the pass that uses the aprons
# up runs whole, its halo follows it on the compute stream, the next pass's
# interior runs beside the halo and only its apron-reading ring waits.
# Expectation: at 16384x32768 (RCCL loopback) the block's exposed time drops
# from ~30 us (ring 35 + halo 48 against a 66 us interior) to under 10 us:
# +5-8 % on the line (68 -> ~72 T); smaller gains at 32768^2 / 32768x65536,
# none at 65536^2.  Parity first (deep-halo + trail + loopback tests).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/o; mkdir -p $O
S=scripts/gpu_step.sh
$S 600 $O/test_trail.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_loopback.py -k "deep_halo or trail or loopback" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/test_trail.log && ! grep -q -E "[0-9]+ (failed|error)" $O/test_trail.log || exit 1
L="python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 96 --warmup 32"
for i in 1 2; do
  for t in 0 1; do
    LIFE_TRAIL_HALO=$t $S 150 $O/loop_16384x32768_t${t}_$i.log $L --shape 16384x32768 || exit $?
  done
done
for sh in 32768x32768 32768x65536 65536x65536; do
  for t in 0 1; do
    LIFE_TRAIL_HALO=$t $S 150 $O/loop_${sh}_t$t.log $L --shape $sh || exit $?
  done
done
for t in 0 1; do
  LIFE_TRAIL_HALO=$t $S 150 $O/loop20_t$t.log python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 20 --warmup 5 || exit $?
  LIFE_TRAIL_HALO=$t $S 300 $O/weak8_t$t.log python -u bench.py --gpus 8 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
$S 150 $O/trace_loop.log timeout -s KILL 140 rocprofv3 --kernel-trace -d $O/trace_loop -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 96 --warmup 32 --shape 16384x32768 || exit $?
echo done
