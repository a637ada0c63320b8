#!/bin/bash
# r05x: thin ring + a CU-masked interior, the mask laid out per XCD.  r05q's
# mask left out the top CU of every 32-bit mask word and the interior ran
# 17 % slower at 65536^2 -- what losing 8 CUs of ONE XCD would cost if CU ids
# interleave over the XCDs (tiles are dealt round-robin to XCDs, so the
# short XCD sets the pace).  Mode 1 leaves out the last 8 ids instead (one
# per XCD if ids interleave).  r05w's trace: the RCCL kernel ran 308 us
# beside the interior (14 us alone).  Expectation: mode 1 costs the interior
# ~3 % (8 of 256 CUs), the halo runs at its own speed, and the 16384x32768
# loopback block shrinks from ~0.106 to ~0.08 ms (+10-15 % on that line).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/x; mkdir -p $O
S=scripts/gpu_step.sh
LIFE_COMM_CUS=1 LIFE_COMM_CUS_MODE=1 $S 600 $O/test_ring.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_loopback.py -k "thin_ring or deep_halo or loopback" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/test_ring.log && ! grep -q -E "[0-9]+ (failed|error)" $O/test_ring.log || exit 1
L="python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 96 --warmup 32"
for sh in 16384x32768 65536x65536 32768x32768; do
  for i in 1 2; do
    $S 150 $O/loop_${sh}_c0_$i.log $L --shape $sh || exit $?
    LIFE_COMM_CUS=1 LIFE_COMM_CUS_MODE=1 $S 150 $O/loop_${sh}_m1_$i.log $L --shape $sh || exit $?
  done
  LIFE_COMM_CUS=1 LIFE_COMM_CUS_MODE=2 $S 150 $O/loop_${sh}_m2.log $L --shape $sh || exit $?
done
LIFE_COMM_CUS=1 LIFE_COMM_CUS_MODE=1 $S 150 $O/loop20_m1.log python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 20 --warmup 5 || exit $?
$S 150 $O/loop20_c0.log python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 20 --warmup 5 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
LIFE_COMM_CUS=1 LIFE_COMM_CUS_MODE=1 $S 150 $O/trace_m1.log timeout -s KILL 140 rocprofv3 --kernel-trace -d $O/trace_m1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 96 --warmup 32 --shape 16384x32768 || exit $?
echo done
