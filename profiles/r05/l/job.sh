#!/bin/bash
# r05l: validation of the round-5 product: smoke, the whole GPU suite, the
# bench lines (driver shape, default, configs[2] 32768^2 bit and byte,
# configs[1] p46gun_big, byte 65536^2, 8 LOCAL shards of 65536^2), the
# RCCL-loopback rehearsals of configs[3]'s per-GPU blocks (the strong-scaling
# prediction, scripts/strong_table.py), rocprofv3 kernel trace + stats of the
# driver-shaped command and of the 32768^2 line, FETCH_SIZE / WRITE_SIZE
# passes of the driver-shaped command.  Expectation: all green; headline
# unchanged (~100 T, 0.45 of VALU); 32768^2 on the dataflow form.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r05/l; mkdir -p $O
S=scripts/gpu_step.sh
$S 120 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
$S 200 $O/bench_driver.log python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
$S 200 $O/bench_default.log python -u bench.py --no-cpu-baseline || exit $?
$S 150 $O/c2_32768.log python -u bench.py --no-cpu-baseline --shape 32768x32768 || exit $?
$S 150 $O/c2_32768_byte.log python -u bench.py --no-cpu-baseline --shape 32768x32768 --kernel byte || exit $?
$S 150 $O/c1_p46.log python -u bench.py --no-cpu-baseline --workload p46gun_big || exit $?
$S 200 $O/bench_byte.log python -u bench.py --no-cpu-baseline --kernel byte || exit $?
$S 300 $O/weak8.log python -u bench.py --gpus 8 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
L="python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 96 --warmup 32"
for sh in 32768x65536 32768x32768 16384x32768 65536x65536; do
  $S 150 $O/loop_$sh.log $L --shape $sh || exit $?
done
$S 150 $O/loop20_65536.log python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 20 --warmup 5 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $R
$S 150 $O/trace_driver.log timeout -s KILL 140 rocprofv3 --kernel-trace --stats -d $O/trace_driver -o run --output-format csv -- python3 $R/bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline || exit $?
$S 150 $O/trace_32768.log timeout -s KILL 140 rocprofv3 --kernel-trace --stats -d $O/trace_32768 -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --shape 32768x32768 || exit $?
$S 90 $O/pmc_fetch.log timeout -s KILL 80 rocprofv3 --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
$S 90 $O/pmc_write.log timeout -s KILL 80 rocprofv3 --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
$S 1100 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
echo done
