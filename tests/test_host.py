"""Host-side logic of the product (no GPU): .cfg loader, VTK writer,
decomposition / dims, layout and the halo plan."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

with open(os.path.join(GOLDEN, "golden.json")) as _f:
    G = json.load(_f)


def test_cfg_loader_matches_reference_frame0(lm):
    for name, rec in G["patterns"].items():
        steps, save, grid = lm.load_cfg(os.path.join(GOLDEN, "cfg", name + ".cfg"))
        assert hashlib.md5(lm.vtk_bytes(grid)).hexdigest() == rec["frames"]["0"][0]


def test_cfg_loader_wraps_and_dedups(lm, tmp_path):
    p = tmp_path / "w.cfg"
    p.write_text("3\n1\n4 3\n0 0\n0 0\n-1 -1\n4 3\n-5 7\n")
    steps, save, g = lm.load_cfg(str(p))
    assert (steps, save, g.shape) == (3, 1, (3, 4))
    want = np.zeros((3, 4), np.uint8)
    want[0, 0] = want[2, 3] = want[1, 3] = 1  # (-1,-1)->(3,2); (4,3)->(0,0); (-5,7)->(3,1)
    np.testing.assert_array_equal(g, want)


def test_cfg_loader_rejects_malformed(lm, tmp_path):
    p = tmp_path / "bad.cfg"
    p.write_text("3\n1\n4 3\n0\n")
    with pytest.raises(ValueError):
        lm.load_cfg(str(p))


@pytest.mark.reference
def test_cfg_loader_vs_reference_loader(lm, oracle):
    import ctypes

    ref = oracle.ref_lib()
    if ref is None:
        pytest.skip("oracle/_ref not built")
    for name in G["patterns"]:
        path = os.path.join(GOLDEN, "cfg", name + ".cfg").encode()
        v = [ctypes.c_int() for _ in range(4)]
        ref.ref_load_cfg(path, *[ctypes.byref(x) for x in v], None)
        grid = np.zeros((v[3].value, v[2].value), np.uint8)
        ref.ref_load_cfg(path, *[ctypes.byref(x) for x in v], grid.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
        steps, save, mine = lm.load_cfg(path.decode())
        assert (steps, save) == (v[0].value, v[1].value)
        np.testing.assert_array_equal(mine, grid)


@pytest.mark.reference
def test_vtk_writer_vs_reference_writer(lm, oracle, tmp_path):
    import ctypes

    ref = oracle.ref_lib()
    if ref is None:
        pytest.skip("oracle/_ref not built")
    g = oracle.fill_random(37, 11, 3, 0.5)
    path = str(tmp_path / "ref.vtk").encode()
    ref.ref_save_vtk(path, 37, 11, g.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
    assert open(path, "rb").read() == lm.vtk_bytes(g)


@pytest.mark.parametrize("n,p", [(10, 3), (500, 4), (7, 7), (65536, 4), (1 << 40, 8)])
def test_decomposition(lm, oracle, n, p):
    blocks = [lm.decomposition(n, p, k) for k in range(p)]
    assert blocks == [oracle.decomposition(n, p, k) for k in range(p)]
    assert blocks[0][0] == 0 and blocks[-1][1] == n
    assert all(blocks[k][1] == blocks[k + 1][0] for k in range(p - 1))


def test_dims_create_matches_mpi(lm):
    # MPI_Dims_create(n, 2) values measured under MPICH plus
    # the balanced-factor rule for others.
    want = {1: (1, 1), 2: (2, 1), 3: (3, 1), 4: (2, 2), 5: (5, 1), 6: (3, 2), 8: (4, 2), 12: (4, 3), 16: (4, 4)}
    for n, d in want.items():
        assert lm.dims_create(n) == d



def test_dims_choose_policies(lm):
    """life_dims_choose: cart = MPI_Dims_create, rows = {1,n}, cols = {n,1},
    auto = row strips once every strip is >= LIFE_AUTO_MIN_STRIP_ROWS tall."""
    for n in (1, 2, 3, 4, 6, 8):
        assert lm.dims_choose(4096, 4096, n, "cart") == lm.dims_create(n)
        assert lm.dims_choose(4096, 4096, n, "rows") == (1, n)
        assert lm.dims_choose(4096, 4096, n, "cols") == (n, 1)
    assert lm.dims_choose(65536, 65536 * 8, 8, "auto") == (1, 8)  # bench weak scaling
    assert lm.dims_choose(65536, 65536, 8, "auto") == (1, 8)      # strong: 8192-row strips
    assert lm.dims_choose(10, 10, 4, "auto") == (2, 2)            # glider: strips too short
    assert lm.dims_choose(500, 500, 8, "auto") == (4, 2)
    assert lm.dims_choose(8192, 8191, 8, "auto") == (4, 2)        # 1023-row strips
    with pytest.raises(lm.LifeError):
        lm.dims_choose(10, 3, 4, "rows")  # empty strips
    with pytest.raises(lm.LifeError):
        lm.dims_choose(10, 10, 0, "cart")
    with pytest.raises(lm.LifeError):
        lm.dims_choose(10, 10, 2, 7)

@pytest.mark.parametrize("kernel", ["byte", "bit"])
@pytest.mark.parametrize("nx,ny,dims", [(1, 1, (1, 1)), (65536, 65536, (1, 1)), (1000, 37, (4, 2)),
                                        (3, 2, (3, 2)), (262144, 131072, (4, 2))])
def test_layout_invariants(lm, kernel, nx, ny, dims):
    for r in range(dims[0] * dims[1]):
        L = lm.layout_query(nx, ny, dims, r, kernel)
        cpu = 128 if kernel == "bit" else 16
        assert L.units == -(-L.w // cpu)
        assert L.pitch % 256 == 0 and L.xoff % 16 == 0
        assert L.pitch >= L.xoff + 16 * L.units + 16  # last unit, apron cell, right extra dword
        assert L.rows == L.h + 2 * L.yapron
        assert (L.x0, L.x0 + L.w) == lm.decomposition(nx, dims[0], r // dims[1])
        assert (L.y0, L.y0 + L.h) == lm.decomposition(ny, dims[1], r % dims[1])


def test_layout_rejects_empty_blocks(lm):
    with pytest.raises(lm.LifeError):
        lm.layout_query(3, 10, (4, 1), 0)


@pytest.mark.parametrize("kernel", ["byte", "bit"])
@pytest.mark.parametrize("nx,ny,dims", [(10, 10, (2, 2)), (500, 500, (4, 2)), (7, 5, (2, 1)), (7, 5, (1, 2)),
                                        (9, 9, (3, 3)), (5, 5, (1, 1)), (100, 3, (4, 3)), (256, 64, (2, 2)),
                                        (512, 80, (4, 2)), (64, 40, (1, 4)), (256, 9, (4, 1))])
def test_halo_plan_is_symmetric(lm, kernel, nx, ny, dims):
    """Every recv has a matching send at the peer: same phase, same kind of
    message and shape, matched in issue order (RCCL p2p semantics), and sends
    go to the Cartesian neighbour whose apron they fill.  Both axes
    partitioned with temporal (K-deep) aprons: ONE phase -- columns, rows and
    the four corner blocks (life_cart.c:257-273) -- instead of columns, then
    rows of width + 2 that carry the corners."""
    world = dims[0] * dims[1]
    plans = {r: lm.halo_plan(nx, ny, dims, r, kernel) for r in range(world)}
    lay = {r: lm.layout_query(nx, ny, dims, r, kernel) for r in range(world)}
    for r, ops in plans.items():
        L = lay[r]
        xa, ya, c0, c1 = L.xapron, L.yapron, L.coords[0], L.coords[1]
        fused = dims[0] > 1 and dims[1] > 1 and L.generations_per_exchange > 1
        kinds = {ph: [(o[1], o[3]) for o in ops if o[0] == ph] for ph in (0, 1)}
        S, R, F = lm.HALO_SEND, lm.HALO_RECV, lm.HALO_FILL
        C, W, X = lm.HALO_COLUMN, lm.HALO_ROW, lm.HALO_CORNER
        if fused:
            assert kinds[1] == []
            assert kinds[0] == [(S, C), (S, C), (R, C), (R, C), (S, W), (S, W), (R, W), (R, W)] + \
                [(S, X)] * 4 + [(R, X)] * 4
        else:
            for ph, what in ((0, C), (1, W)):
                want = [(F, what)] if dims[ph] == 1 else [(S, what), (S, what), (R, what), (R, what)]
                assert kinds[ph] == want
        for o in ops:
            if o[1] != R:
                continue
            peer, ph = o[2], o[0]
            kth = [q for q in ops if q[0] == ph and q[1] == R and q[2] == peer].index(o)
            s_ = [q for q in plans[peer] if q[0] == ph and q[1] == S and q[2] == r][kth]
            P = lay[peer]
            assert (s_[3], s_[6], s_[7]) == (o[3], o[6], o[7])  # same kind of message, cells x rows
            dx = dy = 0
            if o[3] in (C, X):  # x-apron <- the peer's edge columns
                assert o[7] == xa
                assert (o[4], s_[4]) in ((-xa, P.w - xa), (L.w, 0))
                dx = -1 if o[4] < 0 else 1
            if o[3] == W:  # y-apron rows <- the peer's edge rows (padded row = owned + yapron)
                assert o[7] == ya
                assert (o[4], s_[4]) in ((0, P.h), (L.h + ya, ya))
                dy = -1 if o[4] == 0 else 1
            if o[3] == X:  # corner: K rows of the peer's top / bottom edge into the top / bottom apron
                assert o[6] == ya
                assert (o[5], s_[5]) in ((0, P.h), (L.h + ya, ya))
                dy = -1 if o[5] == 0 else 1
            assert tuple(P.coords) == ((c0 + dx) % dims[0], (c1 + dy) % dims[1])

@pytest.mark.parametrize("nx,ny,dims,wide", [(65536, 65536, (1, 1), True), (262144, 131072, (4, 2), True),
                                             (1000, 37, (1, 1), True), (31, 37, (1, 1), False),
                                             (64, 7, (2, 1), True), (500, 500, (2, 1), True),
                                             (63, 9, (2, 1), False), (100, 64, (3, 2), True),
                                             (64, 14, (1, 2), True), (96, 64, (3, 2), True),
                                             (96, 62, (3, 2), True), (96, 30, (3, 2), True)])
def test_temporal_mode_selection(lm, nx, ny, dims, wide):
    """Temporal blocking needs blocks at least one lane column wide (bit: a
    64-cell pair, byte: 32 cells; any width: the right column and apron may
    straddle lane columns) and, on a partitioned y axis, >= K rows."""
    for r in range(dims[0] * dims[1]):
        for kernel in ("bit", "byte"):
            L = lm.layout_query(nx, ny, dims, r, kernel)
            K, xa = lm.TEMPORAL_DEPTH[kernel], lm.TEMPORAL_XAPRON[kernel]
            t = wide and nx // dims[0] >= xa and (dims[1] == 1 or ny // dims[1] >= K)
            assert (L.xapron, L.yapron, L.generations_per_exchange) == ((xa, K, K) if t else (1, 1, 1))
            assert L.rows == L.h + 2 * L.yapron
            if t and kernel == "byte":  # room for the 32-byte right apron and the whole 32-byte word holding its last cell
                assert L.pitch >= L.xoff + 32 * ((L.w + 31) // 32 + 1)


def test_bits_frame_roundtrip(lm, oracle, tmp_path):
    g = oracle.fill_random(37, 11, 4, 0.5)
    p = tmp_path / "f.bits"
    p.write_bytes(lm.bits_bytes(g, 123))
    gen, back = lm.load_bits(str(p))
    assert gen == 123
    np.testing.assert_array_equal(back, g)
    assert p.read_bytes().startswith(b"LIFEBITS 1 37 11 123\n") and len(p.read_bytes()) == 21 + 5 * 11


def test_torch_after_library_is_refused(tmp_path):
    """torch imported AFTER liblife_mi355x.so would map a second
    HIP runtime (double free at exit): the binding refuses it with a clear
    ImportError; torch first, then the library, is fine."""
    import subprocess
    import sys

    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-and-open-mp_amd")
    bad = ("import sys; sys.path.insert(0, %r); import life_mi355x as lm; lm._lib()\n"
           "try:\n    import torch\nexcept ImportError as e:\n    print('refused:', e)\n") % pkg
    r = subprocess.run([sys.executable, "-c", bad], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "refused:" in r.stdout and "second copy" in r.stdout, r.stdout + r.stderr
    good = ("import sys; sys.path.insert(0, %r); import torch; import life_mi355x as lm; lm._lib(); "
            "print(lm.dims_create(8))") % pkg
    r = subprocess.run([sys.executable, "-c", good], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "(4, 2)" in r.stdout, r.stdout + r.stderr


def test_plot_life_against_gpu_count(tmp_path):
    """scripts/plot_life.py (6-cartesian/plot_life.py:4-17): T1/TN against the
    GPU count of each line (times.gpus beside times.txt, or --counts), else the
    reference's 1..N ranks."""
    import subprocess
    import sys

    script = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts", "plot_life.py")
    (tmp_path / "times.txt").write_text("8.0\n4.1\n2.2\n1.25\n")
    (tmp_path / "times.gpus").write_text("1\n2\n4\n8\n")
    r = subprocess.run([sys.executable, script, "times.txt", "out.png"], cwd=tmp_path, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "8 GPU(s): 1.250000 s  speed-up 6.40  efficiency 0.80" in r.stdout
    assert (tmp_path / "out.png").stat().st_size > 1000
    (tmp_path / "times.gpus").unlink()
    r = subprocess.run([sys.executable, script, "times.txt", "out2.png"], cwd=tmp_path, capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0 and "4 GPU(s): 1.250000 s" in r.stdout  # reference convention: line k = k ranks
