#!/bin/bash
# r06d: (1) the tail with banded half tiles only (3/4 tier removed after
# r06c): focused parity; the 16384x32768 block as per-launch tiles (--flow 0)
# against the dataflow form (--flow 1) and against the round-4 library's
# unbanded half tiles, same box.  Expectation: tiles ~84 T > dataflow ~75 T
# (r06c / r06a), r4 lower than HEAD (banded halves).
# (2) VERDICT r5 item 3: the controlled scaling tables -- every per-GPU block
# as an RCCL loopback of the axes its N partitions beside the unpartitioned
# line of the same shape and steps, alternating, twice (scripts/scaling_table.py).
# (3) rocprofv3: driver-shaped kernel trace + stats and FETCH / WRITE passes
# (the round-6 roofline evidence), the 16384x32768 loopback trace.
# (4) the whole GPU suite.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r06/d; mkdir -p $O
S=scripts/gpu_step.sh
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider"
$S 120 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
$S 500 $O/pytest_tail.log $T tests/test_gpu_fullsize.py tests/test_gpu_bench.py -m gpu -k "half_tail or tail_split or driver_shape or single_gpu_line" || exit $?
grep -q " passed" $O/pytest_tail.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest_tail.log || exit 1
U="python -u bench.py --no-cpu-baseline"
L="python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity"
for i in 1 2; do
  $S 150 $O/u992_16384x32768_flow0_$i.log $U --shape 16384x32768 --flow 0 || exit $?
  $S 150 $O/u992_16384x32768_flow1_$i.log $U --shape 16384x32768 --flow 1 || exit $?
  LIFE_MI355X_LIB=$R/build_exp/r4/liblife_mi355x.so $S 150 $O/u992_16384x32768_flow0_r4_$i.log $U --shape 16384x32768 --flow 0 || exit $?
  $S 150 $O/u992_32768x32768_flow0_$i.log $U --shape 32768x32768 --flow 0 || exit $?
  $S 150 $O/u992_32768x32768_flow1_$i.log $U --shape 32768x32768 --flow 1 || exit $?
done
for i in 1 2; do
  $S 120 $O/u20_65536_$i.log $U --steps 20 --warmup 5 || exit $?
  $S 120 $O/l20_65536_x_$i.log $L --steps 20 --warmup 5 --loopback-axes x || exit $?
  $S 120 $O/l20_65536_xy_$i.log $L --steps 20 --warmup 5 --loopback-axes xy || exit $?
  $S 150 $O/u992_65536_$i.log $U || exit $?
  $S 150 $O/l992_65536_x_$i.log $L --loopback-axes x || exit $?
  $S 150 $O/l992_65536_xy_$i.log $L --loopback-axes xy || exit $?
  $S 150 $O/u992_32768x65536_$i.log $U --shape 32768x65536 || exit $?
  $S 150 $O/l992_32768x65536_x_$i.log $L --shape 32768x65536 --loopback-axes x || exit $?
  $S 150 $O/u992_32768x32768_$i.log $U --shape 32768x32768 || exit $?
  $S 150 $O/l992_32768x32768_xy_$i.log $L --shape 32768x32768 --loopback-axes xy || exit $?
  $S 150 $O/l992_16384x32768_xy_$i.log $L --shape 16384x32768 --loopback-axes xy || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd $R
$S 150 $O/trace_driver.log timeout -s KILL 140 rocprofv3 --kernel-trace --stats -d $O/trace_driver -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
$S 90 $O/pmc_fetch.log timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
$S 90 $O/pmc_write.log timeout -s KILL 80 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
$S 150 $O/trace_loop16384.log timeout -s KILL 140 rocprofv3 --kernel-trace --stats -d $O/trace_loop16384 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --shape 16384x32768 --steps 96 --warmup 32 || exit $?
$S 1100 $O/pytest.log $T tests -m gpu || exit $?
grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
echo done
