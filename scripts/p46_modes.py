"""configs[1] (p46gun_big 500^2, 10 000 generations): VGPR- and LDS-resident
small-grid kernels vs the temporally blocked HBM kernel at several tile heights, one
process (the LIFE_TEMPORAL_DEPTH env picks K).  Prints one JSON line per mode."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-and-open-mp_amd"))
import life_mi355x as lm  # noqa: E402

_, _, grid = lm.load_cfg(os.path.join(ROOT, "tests", "golden", "cfg", "p46gun_big.cfg"))
ny, nx = grid.shape
GENS = 10000
modes = [("vgpr", 0), ("lds", 0)] + [("tstep", r) for r in (32, 48)]
for rnd in range(2):
    for name, rows in modes:
        if rows:
            lm.tune_temporal(rows, "bit")
        small = {"vgpr": True, "lds": "lds", "tstep": False}[name]
        with lm.Life(nx, ny, kernel="bit", small_grid=small) as life:
            life.upload(grid)
            life.step(64)
            life.sync()
            t = time.perf_counter()
            life.step(GENS)
            life.sync()
            dt = time.perf_counter() - t
            live = life.live_count()
        print(json.dumps({"mode": name, "rows": rows, "K": os.environ.get("LIFE_TEMPORAL_DEPTH", "default"),
                          "round": rnd, "s": round(dt, 5), "gcells": round(nx * ny * GENS / dt / 1e9, 2),
                          "live": live}), flush=True)
