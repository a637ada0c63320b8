#!/bin/bash
# r04o: why the skewed tiles run 17 % longer per tile: segment length
# (1 / 2 / 4 / 8 tiles per workgroup) and a start stagger of the workgroups.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r04/o; mkdir -p $O
S=scripts/gpu_step.sh
LIFE_SKEW=0 $S 150 $O/base.log python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
for seg in 1 2 4 8; do LIFE_SKEW=1 LIFE_SKEW_SEG=$seg $S 150 $O/seg$seg.log python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?; done
for st in 60 120 250; do LIFE_SKEW=1 LIFE_SKEW_STAGGER=$st $S 150 $O/stag$st.log python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?; done
LIFE_SKEW=0 $S 150 $O/base2.log python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline || exit $?
echo done
