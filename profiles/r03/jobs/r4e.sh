#!/bin/bash
# r4e: pair tiles with m = 14 (flow from 4 passes), dispatch-stamped timing events, polled sync:
# GPU suite, bench lines (3 driver-shaped runs), driver-shape trace
set -o pipefail
O=gpurun_out/r4e; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -4 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2 3; do timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_driver_$i.json 2> $O/bench_driver.err || exit 1; done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err && head -c 250 $O/bench_driver.json && echo
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err && head -c 250 $O/bench_default.json && echo
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 120 rocprofv3 --kernel-trace --hip-trace --output-format csv -d $O/trace -o drv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/trace_bench.json 2> $O/trace.err
