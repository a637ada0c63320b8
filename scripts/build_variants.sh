#!/bin/bash
# Experimental builds of liblife_mi355x.so from other git revisions, into
# build_exp/<name>/ (A/B against the working tree in ONE GPU job: bench.py and
# the tests load one through LIFE_MI355X_LIB).  Measurement tool only.
#   usage: build_variants.sh name:REV[:DEFINES] [...]     e.g. build_variants.sh base:HEAD~1
#          REV "WT" = the working tree; DEFINES: comma-separated -D macros, e.g. ahead:WT:LIFE_BP_AHEAD=2
set -e
cd "$(dirname "$0")/.."
pids=()
for spec in "$@"; do
    name=${spec%%:*}; rest=${spec#*:}; rev=${rest%%:*}; defs=""
    [ "$rest" != "$rev" ] && defs=$(echo "${rest#*:}" | tr ',' '\n' | sed 's/^/-D/' | tr '\n' ' ')
    d=build_exp/$name; src=$(mktemp -d); mkdir -p $d
    if [ "$rev" = WT ]; then
        mkdir -p "$src/mpi-and-open-mp_amd" && cp -r mpi-and-open-mp_amd/csrc "$src/mpi-and-open-mp_amd/" && cp -r include "$src/"
    else
        git archive "$rev" mpi-and-open-mp_amd/csrc include | tar -x -C "$src"
    fi
    (for f in life_kernels.hip life_dev.hip life_plan.cpp; do
         /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 $defs -I"$src/include" \
             -I"$src/mpi-and-open-mp_amd/csrc" -c "$src/mpi-and-open-mp_amd/csrc/$f" -o "$d/$f.o" &
     done; wait
     /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $d/liblife_mi355x.so $d/*.o \
         -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib && rm -rf "$src") &
    pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
