#!/bin/bash
# r06b: (1) headline drift, attribution: r06a's ABAB put HEAD 2 % behind the
#     round-4 library at the driver shape (0.430 vs 0.4215 ms per launch)
#     with an identical tstep_bit_kernel<24,true,true,8> instruction stream
#     (only the kernarg size differs), so the difference is host-side: the
#     launch geometry (LIFE_TAIL_SPLIT 2, the model, vs round 4's rule 1).
#     r4 / HEAD / HEAD with LIFE_TAIL_SPLIT=1, three interleaved rounds.
#     Expectation: HEAD+rule1 == r4.
# (2) Does any reserve free the RCCL kernel beside a persistent interior?
#     r06a: with 8 slots left free the RCCL kernel still ran ~340-380 us (it
#     needs 4 waves of ~264 VGPRs: a CU holding at most ONE tile workgroup).
#     Kernel traces of the 20-generation 65536^2 loopback with 8 / 32 / 128 /
#     256 / 384 slots reserved.  Expectation: freed only at >= 256 (every CU
#     down to two tiles or fewer), at a large interior cost.
cd "$GRAFT_REPO_ROOT" || exit 1
R=$GRAFT_REPO_ROOT
O=gpurun_out/r06/b; mkdir -p $O
S=scripts/gpu_step.sh
D="python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
for i in 1 2 3; do
  LIFE_MI355X_LIB=$R/build_exp/r4/liblife_mi355x.so $S 120 $O/drv_r4_$i.log $D || exit $?
  $S 120 $O/drv_head_$i.log $D || exit $?
  LIFE_TAIL_SPLIT=1 $S 120 $O/drv_head_tail1_$i.log $D || exit $?
done
cd /tmp && export TMPDIR=/tmp && cd $R
for r in 8 32 128 256 384; do
  LIFE_PERSIST_RESERVE=$r $S 150 $O/trace_res$r.log timeout -s KILL 140 rocprofv3 --kernel-trace -d $O/trace_res$r -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --rank-mode --loopback --no-parity --steps 20 --warmup 5 || exit $?
done
echo done
