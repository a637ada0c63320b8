#!/bin/bash
# Experimental builds of liblife_mi355x.so from other git revisions, into
# build_exp/<name>/ (A/B against the working tree in ONE GPU job: bench.py and
# the tests load one through LIFE_MI355X_LIB).  Measurement tool only.
#   usage: build_variants.sh name:REV [name:REV ...]     e.g. build_variants.sh base:HEAD~1
set -e
cd "$(dirname "$0")/.."
pids=()
for spec in "$@"; do
    name=${spec%%:*}; rev=${spec#*:}
    d=build_exp/$name; src=$(mktemp -d); mkdir -p $d
    git archive "$rev" mpi-and-open-mp_amd/csrc include | tar -x -C "$src"
    (for f in life_kernels.hip life_dev.hip life_plan.cpp; do
         /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I"$src/include" \
             -I"$src/mpi-and-open-mp_amd/csrc" -c "$src/mpi-and-open-mp_amd/csrc/$f" -o "$d/$f.o" &
     done; wait
     /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $d/liblife_mi355x.so $d/*.o \
         -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib && rm -rf "$src") &
    pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
