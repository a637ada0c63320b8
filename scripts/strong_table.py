#!/usr/bin/env python3
"""Predicted strong-scaling efficiency of configs[3] (65536^2 split over
N = 2/4/8 GPUs, MPI_Dims_create blocks {2,1} / {2,2} / {4,2}) from
single-GPU measurements: each GPU's block is rehearsed on
one MI355X as an RCCL loopback line (`bench.py --rank-mode --loopback --shape
WxH`: the block a periodic partition of itself, its halos through RCCL, the
ring / interior / halo schedule of the multi-GPU path), and

    predicted efficiency(N) = rate(block_N) / rate(65536^2, 1 GPU)

with rates in cell-updates/s per GPU (a GPU updates 1/N of the grid).  It
ignores what a loopback cannot show: xGMI latency against the loopback's
on-device copies, and rank skew.

    python3 scripts/strong_table.py ONE_GPU.log LOOP_32768x65536.log LOOP_32768x32768.log LOOP_16384x32768.log
"""
import json
import sys


def line(path):
    with open(path) as f:
        for ln in f:
            if ln.startswith("{"):
                return json.loads(ln)
    raise SystemExit(f"no JSON line in {path}")


def main():
    one = line(sys.argv[1])
    blocks = [(2, "32768x65536"), (4, "32768x32768"), (8, "16384x32768")]
    rows = ["| N | block per GPU | per-GPU rate (loopback) | exposed halo / block | predicted job rate | "
            "predicted efficiency |", "|---|---|---|---|---|---|"]
    base = one["value"]
    for (n, shape), path in zip(blocks, sys.argv[2:5]):
        d = line(path)
        ph = d.get("phases", {})
        exp = f"{ph['exposed_ms']:.3f} / {ph['block_ms']:.3f} ms" if ph else "-"
        rows.append(f"| {n} | {shape} | {d['value'] / 1e3:.1f} T | {exp} | {n * d['value'] / 1e3:.0f} T | "
                    f"{d['value'] / base:.2f} |")
    print(f"1 GPU 65536^2: {base / 1e3:.1f} Tcell-updates/s ({sys.argv[1]})")
    print("\n".join(rows))


if __name__ == "__main__":
    main()
