#!/bin/bash
# r04f: the store-predicate hoist (loop schedule back to r4b's) A/B on one
# box, then the GPU suite and the headline lines.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r04/f; mkdir -p $O
S=scripts/gpu_step.sh
for i in 1 2 3; do
  $S 120 $O/cur_$i.log python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
  LIFE_MI355X_LIB=$R/build_exp/r4b/liblife_mi355x.so $S 120 $O/r4b_$i.log python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
done
$S 900 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
$S 120 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
$S 200 $O/bench_driver.log python -u bench.py --steps 20 --warmup 5 || exit $?
$S 200 $O/bench_default.log python -u bench.py --no-cpu-baseline || exit $?
$S 200 $O/loop20.log python -u bench.py --steps 20 --warmup 5 --rank-mode --loopback --no-cpu-baseline --no-parity || exit $?
$S 200 $O/loop992.log python -u bench.py --rank-mode --loopback --no-cpu-baseline --no-parity || exit $?
$S 200 $O/byte.log python -u bench.py --kernel byte --no-cpu-baseline || exit $?
$S 200 $O/c2_32768.log python -u bench.py --size 32768 --no-cpu-baseline || exit $?
$S 200 $O/p46.log python -u bench.py --workload p46gun_big --no-cpu-baseline || exit $?
echo done
