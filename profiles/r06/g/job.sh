#!/bin/bash
# r06g: validation after r06f (the exchange-pass interior tail measured flat,
# now off by default): smoke, the driver-shaped line, a kernel trace of the
# 16384x32768 RCCL loopback, the whole GPU suite (incl. the interior tail
# both ways).  Expectation: all green.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r06/g; mkdir -p $O
S=scripts/gpu_step.sh
T="python -u -m pytest -x -q --timeout 600 --timeout-method thread -p no:cacheprovider"
$S 120 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
$S 200 $O/bench_driver.log python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $R
$S 150 $O/trace_loop16384.log timeout -s KILL 140 rocprofv3 --kernel-trace --stats -d $O/trace_loop16384 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --shape 16384x32768 --steps 96 --warmup 32 || exit $?
$S 1000 $O/pytest.log $T tests -m gpu || exit $?
grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
echo done
