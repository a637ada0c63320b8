#!/bin/bash
# r2o: loopback (RCCL self-halo) + driver rank-mode tests, full GPU suite, smoke, default bench, loopback benches
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2o
mkdir -p $O
S=scripts/gpu_step.sh
$S 300 $O/pytest_loop.log python -u -m pytest tests/test_gpu_loopback.py tests/test_gpu_golden.py -m gpu -x -v --timeout 120 --timeout-method thread || exit $?
grep -q " passed" $O/pytest_loop.log && ! grep -q -E "[0-9]+ failed" $O/pytest_loop.log || exit 1
$S 1200 $O/pytest.log python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread || exit $?
$S 300 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
$S 300 $O/bench_default.json python -u bench.py || exit $?
$S 300 $O/bench_driver.json python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
$S 300 $O/bench_loop_local.json python -u bench.py --loopback --steps 480 --warmup 32 --no-cpu-baseline || exit $?
$S 300 $O/bench_loop_rccl.json python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 bench.py --rank-mode --loopback --steps 480 --warmup 32 --no-cpu-baseline || exit $?
$S 300 $O/bench_loop_rccl_byte.json python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29532 bench.py --rank-mode --loopback --kernel byte --steps 480 --warmup 32 --no-cpu-baseline || exit $?
