#!/bin/bash
# r04a: smoke, the whole GPU suite (now with the poisoned parity module),
# driver-shaped bench, RCCL-loopback A/B of the stream priorities.
O=gpurun_out/r04/a; mkdir -p $O
S=scripts/gpu_step.sh
$S 120 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
$S 900 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
$S 300 $O/bench_driver.log python -u bench.py --steps 20 --warmup 5 || exit $?
for i in 1 2; do
$S 300 $O/loop_prio1_$i.log python -u bench.py --steps 20 --warmup 5 --rank-mode --loopback --no-cpu-baseline --no-parity || exit $?
LIFE_STREAM_PRIORITY=0 $S 300 $O/loop_prio0_$i.log python -u bench.py --steps 20 --warmup 5 --rank-mode --loopback --no-cpu-baseline --no-parity || exit $?
done
$S 300 $O/strong4.log python -u bench.py --gpus 4 --scaling strong --steps 20 --warmup 5 --no-cpu-baseline || exit $?
LIFE_STREAM_PRIORITY=0 $S 300 $O/strong4_prio0.log python -u bench.py --gpus 4 --scaling strong --steps 20 --warmup 5 --no-cpu-baseline || exit $?
