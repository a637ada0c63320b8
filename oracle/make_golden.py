#!/usr/bin/env python3
"""Generates tests/golden/golden.json from the REFERENCE itself.

Runs only in the build container, where /root/reference is mounted
(`make -C oracle` builds oracle/_ref from the reference sources first).  The
outputs are data (md5s, live counts, bit-packed final frames); no reference
source is copied.

  1. Every .cfg pattern the reference ships (tests/golden/cfg/*.cfg, copies of
     the reference's input data files) is run through the reference's serial
     program 3-life/life2d.c (oracle/_ref/life2d); the md5 and live count of
     every VTK frame it writes are recorded.
  2. The reference's MPI programs (6-cartesian/life_cart.c, 3-life/life_mpi.c,
     built against the image's MPICH) are run on the same patterns at several
     rank counts and checked frame by frame against life2d (the MPI
     decomposition is a pure re-partition of the same arithmetic).
  3. p46gun_big generation 10000 (cfg steps 10001 / save_steps 10000).
  4. Random grids from the build's counter-based generator, stepped by the
     reference's life_step (3-life/life2d.c:104-130) linked through
     oracle/_ref/liblife2d_ref.so: md5 + live count after 1 / 10 / 100
     generations.
"""
from __future__ import annotations

import glob
import hashlib
import json
import os
import shutil
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
import oracle as O  # noqa: E402

REF = "/root/reference"
GOLDEN = os.path.join(ROOT, "tests", "golden")
CFG = os.path.join(GOLDEN, "cfg")
MPIEXEC = "/opt/conda/bin/mpiexec"


def md5(b: bytes) -> str:
    return hashlib.md5(b).hexdigest()


def vtk_cells(path: str) -> np.ndarray:
    with open(path, "rb") as f:
        lines = f.read().split(b"\n")
    nx, ny = (int(v) - 1 for v in lines[4].split()[1:3])
    vals = np.array([int(v) for v in lines[10:10 + nx * ny]], dtype=np.uint8)
    return vals.reshape(ny, nx)


def run_frames(prog: list, cfg_text: str, vtkdir: str, env=None) -> dict:
    """Runs a reference program on cfg_text in a scratch dir -> {frame: (md5, live, path)}."""
    d = tempfile.mkdtemp(prefix="golden_")
    with open(os.path.join(d, "in.cfg"), "w") as f:
        f.write(cfg_text)
    subprocess.run(prog + ["in.cfg"], cwd=d, check=True, stdout=subprocess.DEVNULL, env=env, timeout=3600)
    out = {}
    for p in sorted(glob.glob(os.path.join(d, vtkdir, "life_*.vtk"))):
        k = int(os.path.basename(p)[5:11])
        with open(p, "rb") as f:
            b = f.read()
        out[k] = (md5(b), None, p)
    return d, out


def pattern_goldens(res: dict) -> None:
    life2d = os.path.join(HERE, "_ref", "life2d")
    res["patterns"] = {}
    for cfg in sorted(glob.glob(os.path.join(CFG, "*.cfg"))):
        name = os.path.basename(cfg)[:-4]
        text = open(cfg).read()
        if name == "p46gun_big":
            continue  # 10000 generations, frame 0 only: handled in big_goldens
        d, frames = run_frames([life2d], text, ".")
        rec = {"frames": {}, "last": None}
        last = max(frames)
        for k, (h, _, p) in frames.items():
            g = vtk_cells(p)
            rec["frames"][str(k)] = [h, int(g.sum())]
        g = vtk_cells(frames[last][2])
        rec["last"] = last
        rec["last_packed"] = np.packbits(g, axis=None).tobytes().hex()
        rec["shape"] = list(g.shape)
        res["patterns"][name] = rec
        shutil.rmtree(d)
        print(f"{name}: {len(frames)} frames, last {last} live {int(g.sum())}")


def mpi_crosscheck(res: dict) -> None:
    """Reference MPI programs vs the serial reference, frame by frame."""
    env = dict(os.environ, MPIR_CVAR_NEMESIS_SHM_EAGER_MAX_SZ="1048576")
    checks = []
    cart = os.path.join(HERE, "_ref", "life_cart")
    mpi3 = os.path.join(HERE, "_ref", "life_mpi3")
    if not (os.path.exists(cart) and os.path.exists(MPIEXEC)):
        res["mpi_crosscheck"] = "skipped: MPICH not available"
        return
    # life_cart runs only with both Cartesian dims > 1 under MPICH (self-send
    # deadlock otherwise); its gather is exact only when
    # dims divide nx and ny.
    cases = [(cart, 4, "glider_10x10"), (cart, 4, "conf1"), (cart, 8, "conf1"), (cart, 4, "p46gun"),
             (cart, 8, "big_osc"), (mpi3, 2, "glider_10x10"), (mpi3, 3, "glider_10x10"), (mpi3, 4, "conf1"),
             (mpi3, 8, "p46gun")]
    for prog, np_, name in cases:
        text = open(os.path.join(CFG, name + ".cfg")).read()
        d, frames = run_frames([MPIEXEC, "-n", str(np_), prog], text, "vtk", env=env)
        want = res["patterns"][name]["frames"]
        same = sum(1 for k, v in frames.items() if want.get(str(k), [None])[0] == v[0])
        checks.append({"program": os.path.basename(prog), "np": np_, "cfg": name, "frames": len(frames),
                       "identical_to_life2d": same})
        shutil.rmtree(d)
        print(f"mpi {os.path.basename(prog)} np={np_} {name}: {same}/{len(frames)} identical")
    res["mpi_crosscheck"] = checks


def big_goldens(res: dict) -> None:
    life2d = os.path.join(HERE, "_ref", "life2d")
    text = open(os.path.join(CFG, "p46gun_big.cfg")).read().split("\n")
    text[0], text[1] = "10001", "10000"
    d, frames = run_frames([life2d], "\n".join(text), ".")
    g = vtk_cells(frames[10000][2])
    res["p46gun_big"] = {"frame0_md5": frames[0][0], "gen10000_md5": frames[10000][0],
                         "gen10000_live": int(g.sum()),
                         "gen10000_packed": np.packbits(g, axis=None).tobytes().hex()}
    committed = os.path.join(REF, "4-life", "vtk", "life_000000.vtk")
    if os.path.exists(committed):
        res["p46gun_big"]["reference_committed_frame0_md5"] = md5(open(committed, "rb").read())
    shutil.rmtree(d)
    print("p46gun_big:", res["p46gun_big"]["gen10000_md5"], res["p46gun_big"]["gen10000_live"])


def random_goldens(res: dict) -> None:
    cases = []
    for (nx, ny) in [(1, 1), (1, 7), (2, 2), (3, 5), (17, 3), (63, 65), (64, 64), (127, 129), (256, 256),
                     (1000, 37), (333, 777), (4096, 64), (1024, 1024)]:
        for seed in (1, 2, 3):
            g0 = O.fill_random(nx, ny, seed, 0.5)
            rec = {"nx": nx, "ny": ny, "seed": seed, "density": 0.5, "init_md5": md5(g0.tobytes()),
                   "gens": {}}
            g = g0
            done = 0
            for gens in (1, 10, 100):
                g = O.ref_life_run(g, gens - done)
                done = gens
                rec["gens"][str(gens)] = [md5(g.tobytes()), int(g.sum())]
            cases.append(rec)
    # One larger case (4096^2, 10 generations) for the GPU tests.
    g0 = O.fill_random(4096, 4096, 1, 0.5)
    g = O.ref_life_run(g0, 10)
    cases.append({"nx": 4096, "ny": 4096, "seed": 1, "density": 0.5, "init_md5": md5(g0.tobytes()),
                  "gens": {"10": [md5(g.tobytes()), int(g.sum())]}})
    res["random"] = cases
    print(f"random: {len(cases)} cases")


def main():
    if not os.path.exists(os.path.join(REF, "3-life", "life2d.c")):
        sys.exit("reference not mounted: golden fixtures can only be regenerated in the build container")
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    res = {"generator": "oracle/make_golden.py", "reference": "kekoveca/MPI-and-Open-MP @ /root/reference"}
    pattern_goldens(res)
    mpi_crosscheck(res)
    big_goldens(res)
    random_goldens(res)
    with open(os.path.join(GOLDEN, "golden.json"), "w") as f:
        json.dump(res, f, indent=1, sort_keys=True)
    print("wrote", os.path.join(GOLDEN, "golden.json"))


if __name__ == "__main__":
    main()
