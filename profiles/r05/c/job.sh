#!/bin/bash
# r05c: where the small shards lose.
# 1. per-workgroup timelines of the dataflow launch (items 0..3 of each
#    workgroup: pulled / dependencies met / stored) at 16384x32768, 32768^2,
#    65536^2, and of the per-launch tiles at 16384x32768.  Expectation: the
#    dataflow items at 16384x32768 wait on dependencies or pay an exposed
#    load / store drain per item (flow = tiles there, r05a), which a
#    scheduling simulation with constant item times says should not happen
#    (0.96 utilisation).
# 2. RCCL-loopback lines at 16384x32768 and 32768^2 with 0 / 1 / 2 CUs per XCD
#    kept free of the interior tiles (LIFE_COMM_CUS).  Expectation: if the
#    halo kernels wait for CU slots behind the interior (r03), exposed_ms
#    drops with 1-2 reserved CUs at a ~3 % interior cost.
# 3. rocprofv3 kernel traces of the 16384x32768 loopback line, LIFE_COMM_CUS
#    0 and 2: the order and overlap of ring, pack, RCCL, unpack, interior.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r05/c; mkdir -p $O
S=scripts/gpu_step.sh
W="python -u scripts/wg_trace.py"
L=build_exp/wgt/liblife_mi355x.so
for sh in 16384x32768 32768x32768 65536x65536; do
  WG_TRACE_FLOW=1 WG_TRACE_SHAPE=$sh LIFE_MI355X_LIB=$L $S 120 $O/wgflow_$sh.log $W 120 || exit $?
done
WG_TRACE_SHAPE=16384x32768 LIFE_MI355X_LIB=$L $S 120 $O/wgtiles_16384x32768.log $W 12 || exit $?
B="python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 96 --warmup 32"
for sh in 16384x32768 32768x32768; do
  for k in 0 1 2 0 2; do
    LIFE_COMM_CUS=$k $S 150 $O/loop_${sh}_cus$k.log $B --shape $sh || exit $?
  done
done
$S 150 $O/serial_16384x32768.log $B --shape 16384x32768 --no-overlap || exit $?
cd /tmp && export TMPDIR=/tmp && cd $R
for k in 0 2; do
  LIFE_COMM_CUS=$k $S 150 $O/trace_loop_cus$k.log timeout -s KILL 140 rocprofv3 --kernel-trace --stats -d $O/trace_loop_cus$k -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 96 --warmup 32 --shape 16384x32768 || exit $?
done
echo done
