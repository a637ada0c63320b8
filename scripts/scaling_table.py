#!/usr/bin/env python3
"""Predicted weak (configs[4]) and strong (configs[3]) scaling efficiency
from controlled single-GPU measurements.

Every per-GPU block is rehearsed on one MI355X as an RCCL-loopback line
(`bench.py --rank-mode --loopback --loopback-axes A --shape WxH`: the block a
periodic partition of itself, its halos through RCCL, the ring / interior /
halo schedule of the multi-GPU path), exchanging only the axes its N
partitions (MPI_Dims_create: N = 2 -> {2,1}, x only; N = 4 -> {2,2} and N = 8
-> {4,2}, both), and divided by the UNPARTITIONED line of the same shape with
the same --steps / --warmup, measured on the same box in alternation (ABAB;
means over the repeats):

  weak(N)   = loop(65536^2, axes of N) / unpart(65536^2)
  strong(N) = loop(block_N, axes of N) / unpart(65536^2)
            = [loop(block_N) / unpart(block_N)]   (the exchange)
            x [unpart(block_N) / unpart(65536^2)] (the smaller block's own rate)

with rates per GPU (a GPU updates its block).  What a loopback cannot show --
xGMI latency against the loopback's self-messages, the one-phase exchange
(the loopback keeps the two-phase plan), rank skew -- is not in it.

    python3 scripts/scaling_table.py MANIFEST.json

MANIFEST: {"dir": "profiles/r06/d", "weak": {"20": {"base": [logs], "x": [logs],
"xy": [logs]}, "992": {...}}, "strong": {"base": [logs], "blocks": [{"n": 2,
"shape": "32768x65536", "axes": "x", "loop": [logs], "unpart": [logs]}, ...]}}
"""
import json
import os
import sys

WEAK_AXES = {2: "x", 4: "xy", 8: "xy"}


def line(path):
    with open(path) as f:
        for ln in f:
            if ln.startswith("{"):
                return json.loads(ln)
    raise SystemExit(f"no JSON line in {path}")


def mean_rate(d, logs):
    vals = [line(os.path.join(d, p))["value"] for p in logs]
    return sum(vals) / len(vals), vals


def exposure(d, logs):
    ph = [line(os.path.join(d, p)).get("phases") for p in logs]
    ph = [p for p in ph if p]
    if not ph:
        return "-"
    e = sum(p["exposed_ms"] for p in ph) / len(ph)
    b = sum(p["block_ms"] for p in ph) / len(ph)
    return f"{e:.3f} / {b:.3f} ms"


def tables(man, root="."):
    d = os.path.join(root, man["dir"])
    out = ["Weak scaling (configs[4]: a 65536^2 block per GPU)", "",
           "| steps | N | axes exchanged | unpartitioned | loopback | exposed halo / block | predicted efficiency |",
           "|---|---|---|---|---|---|---|"]
    eff = {"weak": {}, "strong": {}}
    for steps, w in sorted(man["weak"].items(), key=lambda kv: int(kv[0])):
        base, _ = mean_rate(d, w["base"])
        for n, ax in WEAK_AXES.items():
            if ax not in w:
                continue
            lr, _ = mean_rate(d, w[ax])
            e = lr / base
            eff["weak"][(int(steps), n)] = round(e, 3)
            out.append(f"| {steps} | {n} | {ax} | {base / 1e3:.1f} T | {lr / 1e3:.1f} T | {exposure(d, w[ax])} | "
                       f"{e:.3f} |")
    s = man["strong"]
    base, _ = mean_rate(d, s["base"])
    out += ["", f"Strong scaling (configs[3]: 65536^2 split over N GPUs; 1 GPU: {base / 1e3:.1f} T)", "",
            "| N | block per GPU (axes) | unpartitioned block | loopback block | exchange factor | block-size factor | "
            "predicted efficiency | predicted job rate |", "|---|---|---|---|---|---|---|---|"]
    for b in s["blocks"]:
        lr, _ = mean_rate(d, b["loop"])
        ur, _ = mean_rate(d, b["unpart"])
        e = lr / base
        eff["strong"][b["n"]] = round(e, 3)
        out.append(f"| {b['n']} | {b['shape']} ({b['axes']}) | {ur / 1e3:.1f} T | {lr / 1e3:.1f} T | {lr / ur:.3f} | "
                   f"{ur / base:.3f} | {e:.3f} | {b['n'] * lr / 1e3:.0f} T |")
    return "\n".join(out), eff


def main():
    man = json.load(open(sys.argv[1]))
    txt, _ = tables(man, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    print(txt)


if __name__ == "__main__":
    main()
