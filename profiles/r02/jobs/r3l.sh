#!/bin/bash
# r3l: byte dataflow with line-contiguous loads too: byte flow parity/census, WRITE_SIZE, A/B vs byte tiles
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r3l
mkdir -p $O
S=scripts/gpu_step.sh
R=$GRAFT_REPO_ROOT
$S 300 $O/pytest.log python -u -m pytest tests/test_gpu_flow.py -m gpu -x -q --timeout 200 --timeout-method thread || exit $?
grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
$S 120 $O/pmc_WRITE_SIZE_flow.log timeout -s KILL 100 env LIFE_FLOW_BYTE=1 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_WRITE_SIZE_flow -o run --output-format csv -- python3 $R/bench.py --kernel byte --steps 128 --warmup 32 --no-cpu-baseline || exit $?
for round in 1 2; do
  for F in 1 0; do
    $S 200 $O/byte_f${F}_65536_$round.json env LIFE_FLOW_BYTE=$F python -u bench.py --kernel byte --steps 480 --warmup 32 --no-cpu-baseline || exit $?
    $S 200 $O/byte_f${F}_32768_$round.json env LIFE_FLOW_BYTE=$F python -u bench.py --kernel byte --size 32768 --steps 480 --warmup 32 --no-cpu-baseline || exit $?
  done
done
