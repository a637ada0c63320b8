"""CPU oracle for the Game-of-Life hot path -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s cpu_baseline
leg may import this module, and only as the checker (or the timed CPU
baseline).  The product path (``life_mi355x`` + ``liblife_mi355x.so``) never
imports it.

Two independent restatements of the reference rule live here:

* ``liblife_oracle.so`` (``life_oracle.c``): a C loop restatement of
  ``3-life/life2d.c:104-130`` / ``6-cartesian/life_cart.c:189-215``;
* ``np_life_step``: a numpy ``roll`` restatement of the same rule.

Both are pinned by tests/golden (frames produced by the reference's own
``life2d`` program and by the reference ``life_step`` linked through
``oracle/_ref/liblife2d_ref.so``).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
_REF = None

_u8p = ctypes.POINTER(ctypes.c_uint8)
_i64 = ctypes.c_int64


def build() -> None:
    """Compile liblife_oracle.so (and oracle/_ref when /root/reference exists)."""
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    """The C restatement, built on first use."""
    global _LIB
    if _LIB is None:
        path = os.path.join(HERE, "liblife_oracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        L.oracle_life_step.argtypes = [_i64, _i64, _u8p, _u8p]
        L.oracle_life_step_block.argtypes = [_i64, _i64, _u8p, _u8p, _i64, _i64, _i64, _i64]
        L.oracle_step_padded.argtypes = [_i64, _i64, _i64, _u8p, _u8p]
        L.oracle_life_run.argtypes = [_i64, _i64, _u8p, _i64, ctypes.c_int]
        L.oracle_splitmix64.argtypes = [ctypes.c_uint64]
        L.oracle_splitmix64.restype = ctypes.c_uint64
        L.oracle_fill_random.argtypes = [_i64, _i64, ctypes.c_uint64, ctypes.c_uint32, _u8p]
        L.oracle_fill_random_window.argtypes = [_i64, _i64, _i64, _i64, _i64, ctypes.c_uint64, ctypes.c_uint32,
                                                _u8p]
        L.oracle_decomposition.argtypes = [_i64, ctypes.c_int, ctypes.c_int,
                                           ctypes.POINTER(_i64), ctypes.POINTER(_i64)]
        L.oracle_dims_create.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        L.oracle_live_count.argtypes = [_i64, _u8p]
        L.oracle_live_count.restype = _i64
        _LIB = L
    return _LIB


def ref_lib():
    """The REFERENCE's life2d.c linked via ref_harness.c, or None if not built
    (it exists only where /root/reference was mounted at build time)."""
    global _REF
    if _REF is None:
        path = os.path.join(HERE, "_ref", "liblife2d_ref.so")
        if not os.path.exists(path):
            return None
        L = ctypes.CDLL(path)
        L.ref_life_run.argtypes = [ctypes.c_int, ctypes.c_int, _u8p, ctypes.c_int]
        L.ref_load_cfg.argtypes = [ctypes.c_char_p] + [ctypes.POINTER(ctypes.c_int)] * 4 + [_u8p]
        L.ref_save_vtk.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_int, _u8p]
        _REF = L
    return _REF


def _p(a: np.ndarray):
    assert a.dtype == np.uint8 and a.flags.c_contiguous
    return a.ctypes.data_as(_u8p)


# ---------------------------------------------------------------- C restatement
def life_step(grid: np.ndarray) -> np.ndarray:
    """One generation of a (ny, nx) uint8 periodic grid (life2d.c:104-130)."""
    g = np.ascontiguousarray(grid, dtype=np.uint8)
    out = np.empty_like(g)
    lib().oracle_life_step(g.shape[1], g.shape[0], _p(g), _p(out))
    return out


def life_run(grid: np.ndarray, gens: int, threads: int = 1) -> np.ndarray:
    g = np.array(grid, dtype=np.uint8, order="C", copy=True)
    lib().oracle_life_run(g.shape[1], g.shape[0], _p(g), gens, threads)
    return g


def step_padded(padded: np.ndarray, w: int, h: int) -> np.ndarray:
    """One generation of an apron-padded block; returns a new padded array
    whose owned cells are updated (apron copied through unchanged)."""
    src = np.ascontiguousarray(padded, dtype=np.uint8)
    out = src.copy()
    lib().oracle_step_padded(w, h, src.shape[1], _p(src), _p(out))
    return out


def fill_random(nx: int, ny: int, seed: int, density: float = 0.5) -> np.ndarray:
    g = np.empty((ny, nx), dtype=np.uint8)
    lib().oracle_fill_random(nx, ny, seed, density_to_thr(density), _p(g))
    return g


def fill_random_window(nx: int, x0: int, y0: int, w: int, h: int, seed: int, density: float = 0.5) -> np.ndarray:
    """fill_random's cells of the w x h window at (x0, y0) of a global
    nx-wide grid (x modulo nx: a band may straddle the x = 0 seam)."""
    g = np.empty((h, w), dtype=np.uint8)
    lib().oracle_fill_random_window(nx, x0, y0, w, h, seed, density_to_thr(density), _p(g))
    return g


def density_to_thr(density: float) -> int:
    return min(int(density * 2.0**32), 0xFFFFFFFF)


def decomposition(n: int, p: int, k: int):
    s, e = _i64(), _i64()
    lib().oracle_decomposition(n, p, k, ctypes.byref(s), ctypes.byref(e))
    return s.value, e.value


def dims_create(n: int):
    d = (ctypes.c_int * 2)()
    lib().oracle_dims_create(n, d)
    return d[0], d[1]


# ---------------------------------------------------------------- numpy restatement
def np_life_step(grid: np.ndarray) -> np.ndarray:
    """Independent numpy restatement: n = sum of the 8 periodic neighbours
    (np.roll wraps exactly like ind()), then the B3/S23 rule of
    life2d.c:117-123."""
    g = grid.astype(np.int32)
    n = np.zeros_like(g)
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            if dx or dy:
                n += np.roll(np.roll(g, -dy, axis=0), -dx, axis=1)
    born = (n == 3) & (g == 0)
    survive = ((n == 3) | (n == 2)) & (g == 1)
    return (born | survive).astype(np.uint8)


def checksum(grid: np.ndarray, x0: int = 0, y0: int = 0, nx: int | None = None) -> int:
    """The definition life_dev_checksum implements (include/life_mi355x.h):
    sum over live cells of mix64(y*nx + x + 1) mod 2^64 (numpy uint64 wraps)."""
    ny_, nx_ = grid.shape
    nx = nx_ if nx is None else nx
    ys, xs = np.nonzero(grid)
    v = ((ys.astype(np.uint64) + np.uint64(y0)) * np.uint64(nx) + xs.astype(np.uint64) + np.uint64(x0)
         + np.uint64(1))
    with np.errstate(over="ignore"):
        t = v * np.uint64(0x9E3779B97F4A7C15)
    return int(np.sum(t ^ (t >> np.uint64(29)), dtype=np.uint64))


# ---------------------------------------------------------------- reference (pinning)
def ref_life_run(grid: np.ndarray, gens: int) -> np.ndarray:
    """The reference's own life_step (3-life/life2d.c:104-130), gens times."""
    L = ref_lib()
    if L is None:
        raise RuntimeError("oracle/_ref not built (reference not mounted)")
    g = np.array(grid, dtype=np.uint8, order="C", copy=True)
    rc = L.ref_life_run(g.shape[1], g.shape[0], _p(g), gens)
    assert rc == 0
    return g
