#!/bin/bash
# r4c: pair tile shape x pass size sweep at 65536^2 (default and driver-shaped bench lines)
O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 900 python scripts/shape_sweep.py $O/shape_sweep.jsonl
