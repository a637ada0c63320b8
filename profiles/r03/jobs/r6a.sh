#!/bin/bash
# r6a: the LDS pipe's share of the bit generation loop: scripts/ubench_pair with the neighbour fetches
# removed (pair_nf: same VALU, no ds_bpermute) or halved (pair_1bp) against the shipped form (pair_bp).
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r6a
rm -rf $O; mkdir -p $O
S=scripts/gpu_step.sh
for i in 1 2; do
  $S 120 $O/ubench_pair_$i.txt scripts/ubench_pair || exit $?
done
echo done
