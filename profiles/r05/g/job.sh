#!/bin/bash
# r05g: the one-phase exchange (columns, rows and the four K x xapron corner
# blocks in ONE RCCL group, corners packed / unpacked with the columns) for
# shards partitioned on both axes.  Expectation: the halo chain at
# 16384x32768 loses one RCCL kernel and its gap (~18 of 52 us, r05e trace);
# RCCL-loopback lines +3-6 % at the small shapes.  Then the whole GPU suite
# (the plan change touches every 2-D partition, LOCAL and RCCL).
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r05/g; mkdir -p $O
S=scripts/gpu_step.sh
B="python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 96 --warmup 32"
for sh in 16384x32768 32768x32768 32768x65536 65536x65536; do
  $S 150 $O/loop_$sh.log $B --shape $sh || exit $?
done
$S 150 $O/loop20_65536.log python -u bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 20 --warmup 5 || exit $?
cd /tmp && export TMPDIR=/tmp && cd $R
$S 150 $O/trace_loop.log timeout -s KILL 140 rocprofv3 --kernel-trace -d $O/trace_loop -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 96 --warmup 32 --shape 16384x32768 || exit $?
$S 1100 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
echo done-g
# (r05f's flow cost attribution, which found no box, and the byte 64-row tile)
bash profiles/r05/f/job.sh || exit $?
B2="python -u bench.py --no-cpu-baseline --kernel byte"
for r in 48 64 48 64; do
  LIFE_TEMPORAL_ROWS_BYTE=$r $S 150 $O/byte_r${r}_65536.log $B2 --steps 96 --warmup 32 || exit $?
done
for r in 48 64; do
  LIFE_TEMPORAL_ROWS_BYTE=$r $S 150 $O/byte_r${r}_32768.log $B2 --shape 32768x32768 --steps 96 --warmup 32 || exit $?
done
echo done2
