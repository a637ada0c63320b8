#!/bin/bash
# r2l: GPU suite after the ghost-depth split; defaults at 65536^2 (bit, byte), 32768^2, driver shape
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2l
mkdir -p $O
S=scripts/gpu_step.sh
$S 1200 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread || exit $?
B="python -u bench.py --no-cpu-baseline"
$S 120 $O/bit.json $B --steps 480 --warmup 48 || exit $?
$S 120 $O/byte.json $B --kernel byte --steps 480 --warmup 48 || exit $?
$S 120 $O/bit32768.json $B --size 32768 --steps 480 --warmup 48 || exit $?
$S 120 $O/byte32768.json $B --kernel byte --size 32768 --steps 480 --warmup 48 || exit $?
$S 120 $O/driver.json $B --steps 20 --warmup 5 || exit $?
$S 300 $O/default.json python -u bench.py || exit $?
