"""Partition shape vs per-shard cost, measured on one GPU: P logical shards of
S x S cells each (LOCAL transport, the same layouts, ring/interior regions,
pack/unpack and halo plan the RCCL path runs), every factorisation
d0 x d1 = P.  Time per shard-generation against the 1-shard run shows what a
partition shape costs the GPU that owns one block (the transport itself is
a device copy here, so xGMI latency is not in these numbers).
Prints one JSON line per (kernel, dims)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-and-open-mp_amd"))
import life_mi355x as lm  # noqa: E402

p = argparse.ArgumentParser()
p.add_argument("--size", type=int, default=32768)
p.add_argument("--gens", type=int, default=128)
p.add_argument("--shards", default="1,2,4,8")
p.add_argument("--kernels", default="bit,byte")
a = p.parse_args()


def factorizations(n):
    return [(d, n // d) for d in range(1, n + 1) if n % d == 0]


for kernel in a.kernels.split(","):
    for P in [int(x) for x in a.shards.split(",")]:
        for d0, d1 in factorizations(P):
            nx, ny = a.size * d0, a.size * d1
            with lm.Life(nx, ny, shards=P, kernel=kernel, dims=(d0, d1), transport=lm.XPORT_LOCAL) as life:
                life.fill_random(1, 0.5)
                life.step(64)
                life.sync()
                t = time.perf_counter()
                life.step(a.gens)
                life.sync()
                dt = time.perf_counter() - t
                lay = life.layout()
            per = dt / (a.gens * P) * 1e3
            print(json.dumps({"kernel": kernel, "shards": P, "dims": [d0, d1], "size": a.size,
                              "K": lay.generations_per_exchange, "ms_per_shard_gen": round(per, 5),
                              "gcells": round(nx * ny * a.gens / dt / 1e9, 1)}), flush=True)
