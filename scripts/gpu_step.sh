#!/bin/bash
# Runs one GPU step under its own time limit; stops the whole call on a fault,
# abort, segfault or timeout (exit codes 124/134/137/139 or >128).
# usage: gpu_step.sh SECONDS LOGFILE cmd...
t=$1; log=$2; shift 2
timeout -k 10 "$t" "$@" > "$log" 2>&1
rc=$?
echo "[gpu_step] rc=$rc: $*" | tee -a "$log"
if [ $rc -ge 124 ]; then echo "[gpu_step] fatal rc=$rc, stopping" ; exit $rc; fi
exit 0
