#!/bin/bash
# Experimental builds of liblife_mi355x.so with build-time switches, into
# build_exp/<name>/ (loaded by scripts/tune.py through LIFE_MI355X_LIB).
set -e
cd "$(dirname "$0")/.."
P=mpi-and-open-mp_amd
build() {  # name, extra flags
    local d=build_exp/$1; mkdir -p $d
    for f in life_kernels.hip life_dev.hip life_plan.cpp; do
        /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Iinclude -I$P/csrc $2 -c $P/csrc/$f -o $d/$f.o &
    done
    wait
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o $d/liblife_mi355x.so $d/*.o -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
}
for v in "$@"; do
    case $v in
        hsum0) build hsum0 -DLIFE_HSUM_MODE=0 ;;
        hsum1) build hsum1 -DLIFE_HSUM_MODE=1 ;;
        hsum2) build hsum2 -DLIFE_HSUM_MODE=2 ;;
        hsum3) build hsum3 -DLIFE_HSUM_MODE=3 ;;
        nw16) build nw16 -DLIFE_STACK_WAVES=16 ;;
        nw4) build nw4 -DLIFE_STACK_WAVES=4 ;;
        xcd) build xcd -DLIFE_XCD_ORDER=1 ;;
        drift0) build drift0 -DLIFE_DRIFT=0 ;;
        drift2) build drift2 -DLIFE_DRIFT=2 ;;  # drifting frame for both encodings
        *) echo "unknown variant $v"; exit 1 ;;
    esac
done
