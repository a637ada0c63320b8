#!/bin/bash
# r05b: validation after the round-5 cleanup (skew / reorder / timing-only
# switches removed, tile shapes trimmed, deep-halo option no longer
# exchanges): smoke, the whole GPU suite (now with the configs[2]
# 1000-generation oracle band test and the poisoned deep-halo tests), the
# driver-shaped bench line.  Expectation: all green, headline unchanged.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/b; mkdir -p $O
S=scripts/gpu_step.sh
$S 120 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
$S 1100 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider --durations=15 || exit $?
grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
$S 200 $O/bench_driver.log python -u bench.py --gpus 1 --steps 20 --warmup 5 || exit $?
echo done
