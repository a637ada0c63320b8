#!/bin/bash
# r05xa: per-XCD queues for the dataflow tiles (LIFE_FLOW_XCD): workgroup b
# pulls from queue b % 8, whose items are one contiguous band of tile-row
# groups, so an XCD's tiles share their ghost rows in its own L2.  r05z: the
# dataflow call reads 1.43x the compulsory bytes (one global queue puts
# neighbouring tiles on different XCDs); r05m: its items wait ~3 % more than
# per-launch tiles.  Expectation: reads ~1.1x, 32768^2 +1-3 % (97 -> ~99 T).
# Dataflow parity first (every test that runs the dataflow form).
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r05/xa; mkdir -p $O
S=scripts/gpu_step.sh
$S 600 $O/test_flow.log python -u -m pytest tests/test_gpu_flow.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py -k "flow or temporal_single_shard or c3_1000" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/test_flow.log && ! grep -q -E "[0-9]+ (failed|error)" $O/test_flow.log || exit 1
for i in 1 2; do
  for x in 0 1; do
    LIFE_FLOW_XCD=$x $S 150 $O/c2_x${x}_$i.log python -u bench.py --no-cpu-baseline --shape 32768x32768 || exit $?
  done
done
for x in 0 1; do
  LIFE_FLOW_XCD=$x $S 150 $O/c3n2_x$x.log python -u bench.py --no-cpu-baseline --shape 32768x65536 || exit $?
  LIFE_FLOW_XCD=$x $S 200 $O/f65536_x$x.log python -u bench.py --no-cpu-baseline --flow 1 || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd $R
for c in FETCH_SIZE WRITE_SIZE; do
  $S 90 $O/pmc_${c}.log timeout -s KILL 80 rocprofv3 --pmc $c -d $O/pmc_${c} -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --shape 32768x32768 --steps 96 --warmup 32 || exit $?
done
echo done
