#!/bin/bash
# r05k: (1) dataflow items pull the next item when they start (the atomic's
# 1-3 us round trip hidden behind the dependency poll instead of on every
# item's path), A/B against the previous build (build_exp/prev = HEAD:
# permutes one row ahead only).  Expectation: +2-5 % on the dataflow lines;
# 32768^2 past 0.43 of VALU.  Also generations per pass 10/14 for the
# dataflow form at 32768^2.  (2) RCCL loopback at 16384x32768 with 0/1/2
# CUs per XCD kept from the interior (LIFE_COMM_CUS) under the round-5
# schedule (the halo kernels now queue behind the ring in the compute
# stream).  Flow parity tests first.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r05/k; mkdir -p $O
S=scripts/gpu_step.sh
$S 400 $O/test_flow.log python -u -m pytest tests/test_gpu_flow.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/test_flow.log && ! grep -q -E "[0-9]+ (failed|error)" $O/test_flow.log || exit 1
B="python -u bench.py --no-cpu-baseline --flow 1"
for sh in 32768x32768 16384x32768 32768x65536 65536x65536; do
  $S 120 $O/new_$sh.log $B --shape $sh || exit $?
  LIFE_MI355X_LIB=build_exp/prev/liblife_mi355x.so $S 120 $O/prev_$sh.log $B --shape $sh || exit $?
  $S 120 $O/new2_$sh.log $B --shape $sh || exit $?
done
for m in 10 14; do
  LIFE_BLOCK_GENS=$m $S 120 $O/m${m}_32768.log $B --shape 32768x32768 || exit $?
done
L="python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 96 --warmup 32 --shape 16384x32768"
for k in 0 1 2 0; do
  LIFE_COMM_CUS=$k $S 150 $O/loop_cus$k.log $L || exit $?
done
echo done
