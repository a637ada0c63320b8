"""configs[1] (p46gun_big 500^2, 10 000 generations): the one-workgroup VGPR
kernel vs the same kernel windowed over several CUs (strip height R, K halo
rows, K generations per launch).  One process; one JSON line per mode."""
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
SETS = {"wide": ((1, 8), (1, 16), (1, 24), (2, 8), (2, 16), (2, 24), (2, 32), (3, 16), (3, 32), (4, 32), (4, 48),
                 (6, 64), (8, 64)),
        "deep": ((1, 20), (1, 24), (1, 26), (1, 28), (1, 29), (1, 30), (1, 31), (2, 40), (2, 48), (2, 56), (2, 60),
                 (2, 63))}
modes = [("vgpr", None)] + [("window", rk) for rk in SETS[sys.argv[1] if len(sys.argv) > 1 else "wide"]]
for rnd in range(2):
    for name, rk in modes:
        small = True if name == "vgpr" else "window"
        with lm.Life(nx, ny, kernel="bit", small_grid=small, window=rk) as life:
            life.upload(grid)
            life.step(64)
            life.sync()
            t = time.perf_counter()
            life.step(GENS)
            life.sync()
            dt = time.perf_counter() - t
            live = life.live_count()
        print(json.dumps({"mode": name, "R_K": rk, "round": rnd, "s": round(dt, 5),
                          "gcells": round(nx * ny * GENS / dt / 1e9, 2), "live": live}), flush=True)
