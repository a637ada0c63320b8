#!/bin/bash
# r5c (part A): validation at the working tree (XCD order for bit + byte tiles, bit one-generation depth 18):
# smoke + the whole GPU suite, one-generation XCD order A/B, the bench lines, rocprofv3 stats and
# trace of the default and driver-shaped runs, PMC traffic + SQ of the driver-shaped launch.
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${RUN:-r5c}
mkdir -p $O
S=scripts/gpu_step.sh
R=$GRAFT_REPO_ROOT
$S 300 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
grep -q "smoke ok" $O/smoke.log || exit 1
$S 900 $O/pytest.log python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider || exit $?
tail -2 $O/pytest.log; grep -q " passed" $O/pytest.log && ! grep -q -E "[0-9]+ (failed|error)" $O/pytest.log || exit 1
$S 300 $O/stress.log python -u scripts/stress_small.py 60 || exit $?
grep -q "done bad=0" $O/stress.log || exit 1
echo done
