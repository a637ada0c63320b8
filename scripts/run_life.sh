#!/bin/bash
# run_life.sh -- the reference's benchmark loop (3-life/run_life.sh:3-6,
# job_life.sh:7-8: `mpirun -np i ./life cfg >> times.txt` for i = 1..N) over
# GPU counts: one line of elapsed seconds per run, appended to times.txt in the
# current directory (the reference's format), and the GPU count of each line
# to times.gpus, which scripts/plot_life.py turns into the speed-up plot.
#   scripts/run_life.sh CFG [MAX_GPUS] [extra driver args...]
set -e
cfg=${1:?usage: run_life.sh CFG [MAX_GPUS] [driver args]}
max=${2:-8}
shift $(( $# >= 2 ? 2 : 1 ))
here=$(cd "$(dirname "$0")/.." && pwd)
drv=$here/mpi-and-open-mp_amd/driver/life_mi355x
for ((n = 1; n <= max; n *= 2)); do
    "$drv" "$cfg" --gpus "$n" "$@" >> times.txt
    echo "$n" >> times.gpus
done
