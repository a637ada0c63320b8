#!/bin/bash
# Experimental builds of liblife_mi355x.so that differ only in build-time
# switches of the sweep kernel (csrc/life_sweep.hip), into build_exp/<name>/;
# bench.py / scripts load one through LIFE_MI355X_LIB.  The other objects come
# from the product build (make -C mpi-and-open-mp_amd).
#   usage: build_variants.sh name:FLAGS [name:FLAGS ...]
#   e.g.   build_variants.sh g2:-DLIFE_SWEEP_GROUP=2 dpp:-DLIFE_SWEEP_LEFT=1
set -e
cd "$(dirname "$0")/.."
P=mpi-and-open-mp_amd
make -s -C $P
pids=()
for spec in "$@"; do
    name=${spec%%:*}; flags=${spec#*:}
    d=build_exp/$name; mkdir -p $d
    (/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -I$P/csrc ${flags//,/ } \
        -c $P/csrc/life_sweep.hip -o $d/life_sweep.hip.o &&
     /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $d/liblife_mi355x.so $d/life_sweep.hip.o \
        $P/build/life_kernels.hip.o $P/build/life_dev.hip.o $P/build/life_plan.cpp.o \
        -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib) &
    pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
