#!/bin/bash
# r4a: round-3 validation of the verdict/advice fixes (gather plan + bounded
# waits, single-device ncclCommInitAll loopback, weak default cart, flow
# chunking, 65536^2 band vs oracle) -- full GPU suite, then the two bench shapes.
set -o pipefail
O=gpurun_out/r4a; mkdir -p $O
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -5 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err && cat $O/bench_driver.json | head -c 400 && echo
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_default.json 2> $O/bench_default.err && head -c 300 $O/bench_default.json && echo
