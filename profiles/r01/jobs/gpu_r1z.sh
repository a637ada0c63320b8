#!/bin/bash
# Partition shape vs per-shard cost (LOCAL shards on one GPU), 65536^2 per shard.
set -e
cd "$GRAFT_REPO_ROOT"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r1z; mkdir -p $O
S=$R/scripts/gpu_step.sh
$S 400 $O/partition.log python -u scripts/partition_sweep.py --size 65536 --gens 256
cat $O/partition.log
