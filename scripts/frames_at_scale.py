#!/usr/bin/env python3
"""Output path at scale: the driver's frame cost at 32768^2.

The reference collects the grid to one rank and writes a text VTK frame every
save_steps generations inside its timed loop (6-cartesian/life_cart.c:64-75,
159-187).  Here the same driver loop runs three ways on a random 50 % grid:

  none  --no-vtk                     generations only
  vtk   --save-steps S               device-formatted VTK text (2 B per cell)
  bits  --save-steps S --format bits packed frames (1 bit per cell + header)

and reports, per format, the frame bytes, the time the frames add to the run
(frame wall = t_format - t_none), the frame rate in GB/s over that added time,
and how much of the frames' own cost was hidden behind the generations.  The
frame's own cost is measured by a run whose generations are negligible
(--steps S*F with S = 1 between frames would time frames only): `frame_only`
= the same frames with 1 generation between them.  hidden = 1 - added /
frame_only.  Frames go to a scratch directory (page cache of the box's /tmp
or /dev/shm), deleted after each run.

  python scripts/frames_at_scale.py [--n 32768] [--gens 1000] [--save 100] [--dir /dev/shm]
"""
import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "mpi-and-open-mp_amd", "driver", "life_mi355x")


def run(args, where):
    d = tempfile.mkdtemp(dir=where)
    try:
        r = subprocess.run([DRIVER] + args, cwd=d, capture_output=True, text=True, timeout=900)
        if r.returncode != 0:
            raise SystemExit(f"driver failed: {args}\n{r.stderr[-2000:]}")
        written = sum(os.path.getsize(os.path.join(d, "vtk", f)) for f in os.listdir(os.path.join(d, "vtk"))) \
            if os.path.isdir(os.path.join(d, "vtk")) else 0
        return float(r.stdout.strip().splitlines()[-1]), written
    finally:
        shutil.rmtree(d, ignore_errors=True)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=32768)
    p.add_argument("--gens", type=int, default=1000)
    p.add_argument("--save", type=int, default=100)
    p.add_argument("--dir", default="/dev/shm")
    p.add_argument("--kernel", default="bit")
    a = p.parse_args()
    frames = (a.gens + a.save - 1) // a.save
    base = ["--random", "1,0.5", "--nx", str(a.n), "--ny", str(a.n), "--kernel", a.kernel]
    t_none, _ = run(base + ["--steps", str(a.gens), "--no-vtk"], a.dir)
    out = {"n": a.n, "generations": a.gens, "save_steps": a.save, "frames": frames, "kernel": a.kernel,
           "scratch": a.dir, "t_none_s": round(t_none, 4),
           "gcell_updates_per_s_none": round(a.n * a.n * a.gens / t_none / 1e9, 1)}
    for fmt in ("vtk", "bits"):
        extra = ["--format", "bits"] if fmt == "bits" else []
        t, nbytes = run(base + ["--steps", str(a.gens), "--save-steps", str(a.save)] + extra, a.dir)
        # the same frames with 1 generation between them: the frames' own cost
        t_only, _ = run(base + ["--steps", str(frames), "--save-steps", "1"] + extra, a.dir)
        added = max(t - t_none, 0.0)
        out[fmt] = {"t_s": round(t, 4), "bytes": nbytes, "bytes_per_frame": nbytes // frames,
                    "added_s": round(added, 4), "frame_only_s": round(t_only, 4),
                    "frame_GBps_alone": round(nbytes / t_only / 1e9, 2),
                    "frame_GBps_in_run": round(nbytes / added / 1e9, 2) if added > 0 else None,
                    "hidden_frac": round(1.0 - added / t_only, 3) if t_only > 0 else None}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    sys.exit(main())
