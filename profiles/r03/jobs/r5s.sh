#!/bin/bash
# r5s: CUs reserved for the halo stream (LIFE_COMM_CUS) on the RCCL loopback rehearsal: parity with 16
# reserved, A/B 0 / 8 / 16 / 32 at 20 and 992 generations, kernel trace with 16.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r5s
mkdir -p $O
S=scripts/gpu_step.sh
R=$GRAFT_REPO_ROOT
LIFE_COMM_CUS=16 $S 500 $O/pytest.log python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_loopback.py -k "multi_shard or loopback" -x -q --timeout 250 --timeout-method thread -p no:cacheprovider || exit $?
tail -2 $O/pytest.log; grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
for i in 1 2; do
  for c in 0 8 16 32; do
    LIFE_COMM_CUS=$c $S 200 $O/rccl20_c${c}_$i.json python -u bench.py --rank-mode --loopback --steps 20 --warmup 5 --no-cpu-baseline || exit $?
    LIFE_COMM_CUS=$c $S 200 $O/rccl992_c${c}_$i.json python -u bench.py --rank-mode --loopback --no-cpu-baseline || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp && cd $R
LIFE_COMM_CUS=16 $S 200 $O/trace16.log rocprofv3 --kernel-trace -d $O/trace16 -o run --output-format csv -- python3 $R/bench.py --rank-mode --loopback --steps 20 --warmup 5 --no-cpu-baseline || exit $?
echo done
