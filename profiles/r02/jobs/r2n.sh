#!/bin/bash
# r2n: full GPU suite (driver rank mode, resume numbering, window validation), smoke
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r2n
mkdir -p $O
S=scripts/gpu_step.sh
$S 1200 $O/pytest.log python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread || exit $?
$S 300 $O/smoke.log python -u -c "import __graft_entry__ as g; g.smoke()" || exit $?
