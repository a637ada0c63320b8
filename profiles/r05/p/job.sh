#!/bin/bash
# r05p: thin ring for the exchange pass (life::ThinRing): the ring is one row
# of half-height tiles per partitioned y edge and half-height 4-lane bands
# per x edge (a few dozen workgroups, ~half a tile time) instead of whole
# tiles (a whole tile time, 249 workgroups at 16384x32768); the interior a
# sub-grid beside it.  Expectation: the RCCL-loopback block at 16384x32768
# drops from ~0.11 ms (ring 36 us + halo 62 us) to ~0.085 ms (ring ~18 us):
# 68 -> ~73 T; 32768^2 +3-5 %, 65536^2 +1-3 %, the 8-LOCAL-shard weak line
# +2-4 %.  Parity first: thin-ring / deep-halo / loopback / multi-shard tests.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/p; mkdir -p $O
S=scripts/gpu_step.sh
$S 900 $O/test_ring.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_loopback.py -k "thin_ring or deep_halo or loopback or multi_shard" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/test_ring.log && ! grep -q -E "[0-9]+ (failed|error)" $O/test_ring.log || exit 1
L="python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 96 --warmup 32"
for i in 1 2; do
  for t in 0 1; do
    LIFE_THIN_RING=$t $S 150 $O/loop_16384x32768_r${t}_$i.log $L --shape 16384x32768 || exit $?
  done
done
for sh in 32768x32768 32768x65536 65536x65536; do
  for t in 0 1; do
    LIFE_THIN_RING=$t $S 150 $O/loop_${sh}_r$t.log $L --shape $sh || exit $?
  done
done
for t in 0 1; do
  LIFE_THIN_RING=$t $S 150 $O/loop20_r$t.log python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 20 --warmup 5 || exit $?
  LIFE_THIN_RING=$t $S 300 $O/weak8_r$t.log python -u bench.py --gpus 8 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
$S 150 $O/trace_loop.log timeout -s KILL 140 rocprofv3 --kernel-trace -d $O/trace_loop -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 96 --warmup 32 --shape 16384x32768 || exit $?
echo done
