"""The reference's own mpirun CPU path, timed -- TEST INFRASTRUCTURE ONLY.

Build-container tool (``tests/`` and manual runs only; the reference and
``oracle/_ref`` never travel to the GPU box, so bench.py reports the rates
measured here as constants with their provenance).  It runs
``oracle/_ref/life_cart`` -- the reference's ``6-cartesian/life_cart.c``,
compiled unmodified by ``oracle/Makefile`` against the image's MPICH -- under
``mpiexec -n P`` on a random .cfg, exactly as ``3-life/run_life.sh:5`` /
``3-life/job_life.sh:8`` run it, and reads the program's own ``MPI_Wtime``
line (``life_cart.c:62-80``).

That timer also covers the step-0 ``life_collect`` and the step-0 VTK write
(``life_cart.c:65-72``: 2 B per cell of text, seconds at 4096^2).  The
steady-state generation rate is therefore taken from two runs that differ
only in their step count: rate = cells x (G2 - G1) / (t(G2) - t(G1)); both runs
write the same single frame (save_steps > steps).

Constraints of the reference under MPICH (BASELINE.md caveats): life_cart
deadlocks on a blocking self-send unless both Cartesian dims are > 1, so P
must give MPI_Dims_create(P, 2) two factors > 1 (4, 6, 8, 9, 12, 16 ...); halo
messages >= 64 KiB need the nemesis eager limit raised (set below).
"""
from __future__ import annotations

import os
import shutil
import subprocess
import tempfile
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIFE_CART = os.path.join(HERE, "_ref", "life_cart")
MPIEXEC_CANDIDATES = ("/opt/conda/bin/mpiexec", shutil.which("mpiexec") or "")


def mpiexec():
    for m in MPIEXEC_CANDIDATES:
        if m and os.access(m, os.X_OK):
            return m
    return None


def available() -> bool:
    return os.access(LIFE_CART, os.X_OK) and mpiexec() is not None


def cfg_body(grid: np.ndarray) -> bytes:
    """The cell lines of the reference's .cfg (life_cart.c:104-109): one "i j"
    line per live cell, i = x (the fast index)."""
    ys, xs = np.nonzero(grid)
    # chunked: formatting 8 M lines at once needs ~1 GB of Python strings
    parts = []
    for s in range(0, xs.size, 1 << 20):
        xc, yc = xs[s:s + (1 << 20)], ys[s:s + (1 << 20)]
        parts.append("".join(f"{x} {y}\n" for x, y in zip(xc.tolist(), yc.tolist())).encode())
    return b"".join(parts)


def write_cfg(path: str, nx: int, ny: int, body: bytes, steps: int, save_steps: int) -> None:
    """The reference's .cfg (life_cart.c:92-98): steps, save_steps, "nx ny", then the cells."""
    with open(path, "wb") as f:
        f.write(f"{steps}\n{save_steps}\n{nx} {ny}\n".encode())
        f.write(body)


def run_once(workdir: str, cfg: str, procs: int, timeout: float) -> float:
    env = dict(os.environ)
    env.setdefault("MPIR_CVAR_NEMESIS_SHM_EAGER_MAX_SZ", "1048576")
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([mpiexec(), "-n", str(procs), LIFE_CART, cfg], cwd=workdir, env=env,
                       capture_output=True, text=True, timeout=timeout)
    if r.returncode != 0:
        raise RuntimeError(f"life_cart np {procs} failed ({r.returncode}): {r.stderr[-400:]}")
    lines = [ln for ln in r.stdout.split() if ln.strip()]
    return float(lines[-1])


def steady_rate(grid: np.ndarray, procs: int, target_s: float = 10.0, probe_gens: int = 20,
                timeout: float = 300.0) -> dict:
    """Steady-state cell-updates/s of the reference life_cart under mpiexec -n
    procs on `grid` (uint8 0/1, ny x nx), about `target_s` of timed
    generations beyond the shared first frame."""
    if not available():
        raise RuntimeError("oracle/_ref/life_cart or mpiexec missing")
    ny, nx = grid.shape
    body = cfg_body(grid)
    work = tempfile.mkdtemp(prefix="life_cart_")
    try:
        def timed(gens: int) -> float:
            cfg = os.path.join(work, f"g{gens}.cfg")
            write_cfg(cfg, nx, ny, body, gens, gens + 1)  # one frame (step 0), `gens` generations
            return run_once(work, cfg, procs, timeout)

        t0 = time.perf_counter()
        t_a = timed(1)
        t_b = timed(1 + probe_gens)
        per_gen = max((t_b - t_a) / probe_gens, 1e-6)
        gens = 1 + probe_gens + max(probe_gens, int(target_s / per_gen))
        t_c = timed(gens)
        wall = time.perf_counter() - t0
    finally:
        shutil.rmtree(work, ignore_errors=True)
    dg = gens - 1
    dt = t_c - t_a
    return {"value": nx * ny * dg / dt / 1e9, "unit": "Gcell-updates/s", "cores": procs, "kind": "reference",
            "sample": f"reference 6-cartesian/life_cart.c (oracle/_ref, gcc -O2, MPICH) under mpiexec -n {procs} "
                      f"on random 50% {nx}x{ny}: steady state from two runs of 1 and {gens} generations "
                      f"({t_a:.2f} s vs {t_c:.2f} s on its MPI_Wtime; the shared step-0 frame write cancels); "
                      f"{wall:.0f} s wall incl. .cfg writes"}
