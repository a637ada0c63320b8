"""Reference file formats: the .cfg pattern loader and the VTK frame writer.

* ``load_cfg`` restates the parsing half of life_init
  (6-cartesian/life_cart.c:92-111): ``steps``, ``save_steps``, ``nx ny``,
  then one live cell ``i j`` per line, coordinates wrapped periodically
  (x = i is the contiguous axis).  Malformed input raises instead of looping
  forever as the reference's fscanf loop does.
* ``save_vtk`` / ``vtk_bytes`` restate life_save_vtk (life_cart.c:159-187):
  ASCII STRUCTURED_POINTS, one ``%d\\n`` per cell, y outer, x inner.
"""
from __future__ import annotations

import os

import numpy as np


def load_cfg(path: str):
    """-> (steps, save_steps, grid[ny, nx] uint8)."""
    with open(path, "r") as f:
        toks = f.read().split()
    try:
        vals = [int(t) for t in toks]
    except ValueError as e:
        raise ValueError(f"{path}: non-integer token: {e}") from None
    if len(vals) < 4 or (len(vals) - 4) % 2:
        raise ValueError(f"{path}: expected 'steps save_steps nx ny' then 'i j' pairs")
    steps, save_steps, nx, ny = vals[:4]
    if nx <= 0 or ny <= 0:
        raise ValueError(f"{path}: bad grid size {nx}x{ny}")
    grid = np.zeros((ny, nx), dtype=np.uint8)
    if len(vals) > 4:
        c = np.asarray(vals[4:], dtype=np.int64).reshape(-1, 2)
        grid[np.mod(c[:, 1], ny), np.mod(c[:, 0], nx)] = 1  # u0[ind(i, j)] = 1
    return steps, save_steps, grid


def vtk_header(nx: int, ny: int) -> bytes:
    return ("# vtk DataFile Version 3.0\n"
            "Created by write_to_vtk2d\n"
            "ASCII\n"
            "DATASET STRUCTURED_POINTS\n"
            f"DIMENSIONS {nx + 1} {ny + 1} 1\n"
            "SPACING 1 1 0.0\n"
            "ORIGIN 0 0 0.0\n"
            f"CELL_DATA {nx * ny}\n"
            "SCALARS life int 1\n"
            "LOOKUP_TABLE life_table\n").encode()


def vtk_bytes(grid: np.ndarray) -> bytes:
    ny, nx = grid.shape
    body = np.empty((ny * nx, 2), dtype=np.uint8)
    body[:, 0] = np.where(grid.reshape(-1) != 0, ord("1"), ord("0"))
    body[:, 1] = ord("\n")
    return vtk_header(nx, ny) + body.tobytes()


def bits_bytes(grid: np.ndarray, generation: int = 0) -> bytes:
    """The driver's packed frame (--format bits): 'LIFEBITS 1 nx ny gen\\n'
    then rows of ceil(nx/8) bytes, cell x at bit x&7 of byte x>>3."""
    ny, nx = grid.shape
    rows = np.packbits(grid.astype(bool), axis=1, bitorder="little")
    return f"LIFEBITS 1 {nx} {ny} {generation}\n".encode() + rows.tobytes()


def load_bits(path: str):
    """-> (generation, grid[ny, nx] uint8) of a --format bits frame."""
    with open(path, "rb") as f:
        head = f.readline().split()
        if len(head) != 5 or head[0] != b"LIFEBITS" or head[1] != b"1":
            raise ValueError(f"{path}: not a LIFEBITS v1 frame")
        nx, ny, gen = int(head[2]), int(head[3]), int(head[4])
        raw = np.frombuffer(f.read(), dtype=np.uint8)
    rb = (nx + 7) // 8
    if raw.size != rb * ny:
        raise ValueError(f"{path}: truncated")
    grid = np.unpackbits(raw.reshape(ny, rb), axis=1, bitorder="little")[:, :nx]
    return gen, np.ascontiguousarray(grid, dtype=np.uint8)


def save_vtk(path: str, grid: np.ndarray) -> None:
    """life_save_vtk: creates ./vtk if missing (life_cart.c:163-166)."""
    if os.path.basename(os.path.dirname(path)) == "vtk" and not os.path.isdir(os.path.dirname(path)):
        os.makedirs(os.path.dirname(path), mode=0o700, exist_ok=True)
    with open(path, "wb") as f:
        f.write(vtk_bytes(grid))
