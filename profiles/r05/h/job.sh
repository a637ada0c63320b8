#!/bin/bash
# r05h: banded dataflow items (the last tile column as bands, as the
# per-launch tiles do) and the automatic dataflow default (LIFE_OPT_FLOW 3:
# the dataflow form when a pass is under 5 rounds of resident workgroups).
# Expectation: 32768^2 (9th tile column owns 16 of 64 lanes) rises from
# 0.4135 (r05a, flow 1) to ~0.43-0.44 of VALU; 16384x32768 (o = 8) gains
# more than that in issued terms.  First the flow parity tests (banded shapes
# added), then the lines, a kernel trace of the 32768^2 line.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r05/h; mkdir -p $O
S=scripts/gpu_step.sh
$S 400 $O/test_flow.log python -u -m pytest tests/test_gpu_flow.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/test_flow.log && ! grep -q -E "[0-9]+ (failed|error)" $O/test_flow.log || exit 1
B="python -u bench.py --no-cpu-baseline"
for sh in 32768x32768 16384x32768 32768x65536; do
  $S 120 $O/auto_$sh.log $B --shape $sh || exit $?
  LIFE_FLOW_BANDS=0 $S 120 $O/nobands_$sh.log $B --shape $sh --flow 1 || exit $?
  $S 120 $O/tiles_$sh.log $B --shape $sh --flow 0 || exit $?
done
$S 120 $O/auto_65536.log $B || exit $?
$S 120 $O/driver_65536.log python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $R
$S 150 $O/trace_32768.log timeout -s KILL 140 rocprofv3 --kernel-trace --stats -d $O/trace_32768 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --shape 32768x32768 || exit $?
echo done
