"""Diagnose the dims (2,1) LOCAL mismatch: smallest failing size and where."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "mpi-and-open-mp_amd"), os.path.join(ROOT, "oracle")]
import numpy as np
import life_mi355x as lm
import oracle as O

for kernel in ("bit",):
    for nx, ny, gens, dims in [(128, 2000, 40, (2, 1)), (4096, 2000, 40, (2, 1)), (8192, 2000, 40, (2, 1)),
                               (8192, 2000, 1, (2, 1)), (8192, 2000, 32, (2, 1)), (8192, 2000, 33, (2, 1)),
                               (8192, 600, 40, (2, 1)), (8192, 2000, 40, (4, 1)), (8192, 2000, 40, (2, 2))]:
        g0 = O.fill_random(nx, ny, 5, 0.5)
        want = O.life_run(g0, gens, threads=8)
        with lm.Life(nx, ny, shards=dims[0] * dims[1], kernel=kernel, dims=dims, transport=lm.XPORT_LOCAL) as life:
            life.upload(g0)
            life.step(gens)
            got = life.gather()
        bad = np.argwhere(got != want)
        print(kernel, nx, ny, gens, dims, "mismatches", len(bad),
              "rows", (bad[:, 0].min(), bad[:, 0].max()) if len(bad) else None,
              "cols", sorted(set((bad[:, 1] // 32).tolist()))[:12] if len(bad) else None, flush=True)
