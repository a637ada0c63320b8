#!/bin/bash
# r5j: automatic dataflow policy (LIFE_OPT_FLOW 3): flow + bench tests, the 32768^2 / 65536^2 default
# lines, and the byte one-generation rows x depth sweep with the XCD strip order.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5j
mkdir -p $O
S=scripts/gpu_step.sh
$S 600 $O/pytest.log python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_bench.py tests/test_gpu_parity.py -x -q --timeout 250 --timeout-method thread -p no:cacheprovider || exit $?
tail -2 $O/pytest.log; grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
for i in 1 2; do
  $S 200 $O/s32768_auto_$i.json python -u bench.py --size 32768 --no-cpu-baseline || exit $?
  $S 200 $O/s32768_tiles_$i.json python -u bench.py --size 32768 --flow 0 --no-cpu-baseline || exit $?
done
$S 200 $O/def.json python -u bench.py --no-cpu-baseline || exit $?
LIFE_TEMPORAL_DEPTH_BYTE=1 $S 300 $O/tune_byte1.log python -u scripts/tune.py --kernels byte --rows 16,32,64 --depths 2,4,8 --gens 10 --rounds 3 || exit $?
echo done
