#!/usr/bin/env python3
"""Sweep of the bit tile shape (pair rows R x waves NW) and the generations per
pass m at 65536^2 (measurement tool): one bench.py process per point, since
the knobs are read at library load (LIFE_TEMPORAL_ROWS, LIFE_TILE_WAVES,
LIFE_BLOCK_GENS).  Writes one JSON line per run to the output file.

  python3 scripts/shape_sweep.py OUT.jsonl [--shapes 24x8,16x16] [--m 10,20] [--modes default,driver]
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MODES = {"default": [], "driver": ["--steps", "20", "--warmup", "5"]}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("out")
    p.add_argument("--shapes", default="24x8,16x8,32x8,24x12,16x16,24x16")
    p.add_argument("--m", default="10,12,16,20")
    p.add_argument("--modes", default="default,driver")
    p.add_argument("--size", default="65536")
    p.add_argument("--extra", default="")
    p.add_argument("--reps", type=int, default=1)
    a = p.parse_args()
    with open(a.out, "a") as f:
        for shape in a.shapes.split(","):
            R, NW = shape.split("x")
            for m in a.m.split(","):
                for mode in [md for md in a.modes.split(",") for _ in range(a.reps)]:
                    env = dict(os.environ, LIFE_TEMPORAL_ROWS=R, LIFE_TILE_WAVES=NW, LIFE_BLOCK_GENS=m)
                    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--size", a.size,
                           *MODES[mode], *a.extra.split()]
                    t = time.time()
                    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
                    line = next((ln for ln in r.stdout.splitlines() if ln.startswith("{")), None)
                    rec = {"R": int(R), "NW": int(NW), "m": int(m), "mode": mode, "size": int(a.size), "rc": r.returncode,
                           "wall_s": round(time.time() - t, 1)}
                    if line:
                        d = json.loads(line)
                        ro = d["roofline"]
                        rec.update(value=d["value"], ms_per_step=d["ms_per_step"], kernel_ms=ro.get("kernel_avg_ms"),
                                   launches=ro.get("kernel_launches"), path=d["config"]["kernel_path"],
                                   frac=ro.get("frac"))
                    else:
                        rec["err"] = r.stderr[-400:]
                    print(json.dumps(rec), flush=True)
                    f.write(json.dumps(rec) + "\n")
                    f.flush()


if __name__ == "__main__":
    main()
