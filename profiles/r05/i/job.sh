#!/bin/bash
# r05i: (1) persistent byte tiles (tpers_byte_kernel: one 16-wave workgroup
# per CU, the next tile's window loaded under the current generations):
# parity first, then 65536^2 / 32768^2 byte lines against LIFE_BYTE_PERSIST=0.
# Expectation: the 33 us load phase per tile (r04 byte_ab) disappears; byte
# 65536^2 from ~68 T towards 80 T, traffic unchanged.
# (2) r05h again (it stopped at the old default-off test after 30 flow parity
# cases passed, banded ones included): banded dataflow items and the
# automatic dataflow default; 32768^2 from 0.4135 (flow 1, r05a) to ~0.43.
# Then the whole GPU suite.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r05/i; mkdir -p $O
S=scripts/gpu_step.sh
$S 300 $O/test_persist.log python -u -m pytest tests/test_gpu_parity.py -k "byte_persistent or temporal_single_shard" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/test_persist.log && ! grep -q -E "[0-9]+ (failed|error)" $O/test_persist.log || exit 1
B="python -u bench.py --no-cpu-baseline"
for p in 1 0 1 0; do
  LIFE_BYTE_PERSIST=$p $S 150 $O/byte_p${p}_65536.log $B --kernel byte || exit $?
done
for p in 1 0; do
  LIFE_BYTE_PERSIST=$p $S 150 $O/byte_p${p}_32768.log $B --kernel byte --shape 32768x32768 || exit $?
done
for sh in 32768x32768 16384x32768 32768x65536; do
  $S 120 $O/auto_$sh.log $B --shape $sh || exit $?
  LIFE_FLOW_BANDS=0 $S 120 $O/nobands_$sh.log $B --shape $sh --flow 1 || exit $?
  $S 120 $O/tiles_$sh.log $B --shape $sh --flow 0 || exit $?
done
$S 120 $O/auto_65536.log $B || exit $?
$S 120 $O/driver_65536.log python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $R
$S 150 $O/trace_32768.log timeout -s KILL 140 rocprofv3 --kernel-trace --stats -d $O/trace_32768 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --shape 32768x32768 || exit $?
$S 150 $O/trace_byte.log timeout -s KILL 140 rocprofv3 --kernel-trace --stats -d $O/trace_byte -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --kernel byte --steps 96 --warmup 32 || exit $?
$S 1100 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
echo done
