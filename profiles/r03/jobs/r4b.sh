#!/bin/bash
# r4b: first run of the interleaved-pair bit layout (pair tiles, R = 24 pair rows x 8 waves):
# smoke, full GPU suite, then the two bench shapes.
set -o pipefail
O=gpurun_out/r4b; mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -3 $O/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -15 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err && head -c 300 $O/bench_driver.json && echo
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err && head -c 300 $O/bench_default.json && echo
