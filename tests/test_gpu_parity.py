"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bit-exact on every cell.  The oracle restates 3-life/life2d.c:104-130 and is
itself pinned to the reference (tests/test_oracle.py).
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SIZES = [(1, 1), (1, 5), (5, 1), (2, 3), (3, 2), (16, 16), (17, 3), (31, 33), (63, 64), (64, 63),
         (65, 65), (127, 5), (128, 128), (129, 130), (200, 1), (1000, 37), (257, 300)]


@pytest.mark.parametrize("small", [False, "lds", True], ids=["stream", "lds", "vgpr"])
@pytest.mark.parametrize("kernel", ["byte", "bit"])
@pytest.mark.parametrize("nx,ny", SIZES)
def test_single_shard(gpu, oracle, kernel, nx, ny, small):
    """stream: the HBM-streaming kernels (one-generation or temporal);
    lds: the LDS-resident small-grid kernel; vgpr: the register-resident one
    where the shape allows it (else LDS)."""
    g0 = oracle.fill_random(nx, ny, seed=nx * 1000 + ny, density=0.4)
    with gpu.Life(nx, ny, shards=1, kernel=kernel, small_grid=small) as life:
        life.upload(g0)
        np.testing.assert_array_equal(life.gather(), g0)
        life.step(1)
        np.testing.assert_array_equal(life.gather(), oracle.life_run(g0, 1))
        life.step(6)
        want = oracle.life_run(g0, 7)
        np.testing.assert_array_equal(life.gather(), want)
        assert life.live_count() == int(want.sum())


@pytest.mark.parametrize("kernel", ["byte", "bit"])
@pytest.mark.parametrize("nx,ny,seed", [(1000, 37, 1), (4096, 64, 2), (333, 777, 3)])
def test_fill_random_matches_oracle(gpu, oracle, kernel, nx, ny, seed):
    with gpu.Life(nx, ny, kernel=kernel) as life:
        life.fill_random(seed, 0.5)
        np.testing.assert_array_equal(life.gather(), oracle.fill_random(nx, ny, seed, 0.5))


@pytest.mark.parametrize("kernel", ["byte", "bit"])
@pytest.mark.parametrize("shards,dims,nx,ny", [
    (2, (0, 0), 100, 40), (4, (0, 0), 65, 33), (8, (0, 0), 300, 130), (6, (0, 0), 47, 29),
    (4, (1, 4), 70, 50), (4, (4, 1), 70, 50), (3, (3, 1), 5, 9), (2, (1, 2), 3, 2),
    (8, (4, 2), 4, 2), (4, (2, 2), 260, 260),
    (8, (1, 8), 64, 320), (4, (1, 4), 96, 132), (2, (1, 2), 300, 70),  # row strips (temporal)
])
@pytest.mark.parametrize("overlap", [True, False], ids=["overlap", "serial"])
def test_multi_shard_local(gpu, oracle, kernel, shards, dims, nx, ny, overlap):
    """P logical shards on one GPU, halo through the LOCAL transport: the same
    plan and pack/unpack kernels the RCCL transport runs; the overlapped
    schedule (ring, interior and halo on three streams) and the serial one
    (LIFE_OPT_OVERLAP 0: all tiles in one launch, then the halo)."""
    g0 = oracle.fill_random(nx, ny, seed=shards * 7 + nx, density=0.45)
    with gpu.Life(nx, ny, shards=shards, kernel=kernel, dims=dims, transport=gpu.XPORT_LOCAL,
                  overlap=overlap) as life:
        life.upload(g0)
        np.testing.assert_array_equal(life.gather(), g0)
        done = 0
        for total in (1, 4, 10):
            life.step(total - done)
            done = total
            want = oracle.life_run(g0, total)
            np.testing.assert_array_equal(life.gather(), want, err_msg=f"generation {total}")
        assert life.live_count() == int(want.sum())


@pytest.mark.parametrize("kernel", ["byte", "bit"])
def test_onegen_wide_interior_local(gpu, oracle, kernel):
    """the overlapped one-generation schedule joins each
    generation into ONE stream, so the next interior must be fenced behind
    everything on the compute stream.  Row strips 24 rows tall (< K: the
    one-generation layout) and 131072 cells wide: each shard's interior (22
    rows) runs far longer than its ring (2 rows) + halo, the shape where a
    missing fence lets two generations' interiors overlap."""
    nx, ny, shards = 131072, 16 * 24, 16
    g0 = oracle.fill_random(nx, ny, seed=5, density=0.5)
    with gpu.Life(nx, ny, shards=shards, kernel=kernel, dims=(1, shards), transport=gpu.XPORT_LOCAL) as life:
        assert life.layout().generations_per_exchange == 1
        life.upload(g0)
        life.step(1)
        np.testing.assert_array_equal(life.gather(), oracle.life_run(g0, 1, threads=8), err_msg="generation 1")
        life.step(9)
        assert life.last_path() == "onegen"
        np.testing.assert_array_equal(life.gather(), oracle.life_run(g0, 10, threads=8), err_msg="generation 10")


@pytest.mark.parametrize("nx", [1024, 1000], ids=["temporal", "onegen"])
def test_byte_equals_bit_long(gpu, oracle, nx):
    ny, gens = 768, 200
    g0 = oracle.fill_random(nx, ny, seed=11, density=0.5)
    out = {}
    for k in ("byte", "bit"):
        with gpu.Life(nx, ny, kernel=k, small_grid=False) as life:
            life.upload(g0)
            life.step(gens)
            out[k] = life.gather()
    np.testing.assert_array_equal(out["byte"], out["bit"])
    np.testing.assert_array_equal(out["bit"], oracle.life_run(g0, gens, threads=4))


@pytest.mark.parametrize("flow", [0, 1], ids=["tiles", "flow"])
@pytest.mark.parametrize("kernel,nx,gens", [("bit", 4096, 72), ("bit", 31, 13), ("bit", 63, 13), ("byte", 4096, 40),
                                            ("byte", 31, 13)])
def test_timing_stats(gpu, kernel, nx, gens, flow):
    """One timed launch per generation (one-generation kernels: a block
    narrower than the x-apron, 64 bit cells / 32 byte cells) or per up to K
    generations (temporal kernels).  Bytes are the compulsory HBM traffic: 0.25 B (bit) / 2 B
    (byte) per cell per LAUNCH; cell-updates are cells x generations; VALU
    lane-ops are modelled for the temporal kernels only.  The dataflow tiles
    (flow, bit: 72 generations = 6 passes of 12) count each of their passes
    as one launch."""
    K = gpu.TEMPORAL_DEPTH[kernel]
    temporal = nx >= gpu.TEMPORAL_XAPRON[kernel]
    # ceil(gens / bmax) launches of nearly equal size, bmax = K capped by
    # BLOCK_GENS (the dataflow passes: gens // bmax of bmax, here exact)
    bmax = min(K, 32, gpu.BLOCK_GENS[kernel])
    sizes, left = [], gens
    while temporal and left:
        n = -(-left // bmax)
        sizes.append(-(-left // n))
        left -= sizes[-1]
    launches = len(sizes) if temporal else gens
    with gpu.Life(nx, 4096, kernel=kernel, small_grid=False, flow=flow) as life:
        life.fill_random(1)
        life.set_timing(True)
        life.step(gens)
        assert life.last_path() == ("flow" if flow and kernel == "bit" and temporal else
                                    "tiles" if temporal else "onegen")
        ms, n, b = life.kernel_stats()
        upd, valu = life.kernel_work()
        assert n == launches and ms > 0
        assert n * b == pytest.approx(nx * 4096 * launches * (0.25 if kernel == "bit" else 2.0))
        assert n * upd == pytest.approx(nx * 4096 * gens)
        assert (valu > 0) == temporal
        if temporal:  # ceil(4096 / (NW waves x R rows - 2m)) tile rows of 62-lane tiles, 64 lanes each
            R, NW = gpu.TEMPORAL_ROWS[kernel], gpu.TILE_WAVES[kernel]
            if kernel == "bit" and os.environ.get("LIFE_TEMPORAL_ROWS") == "16":
                R = int(os.environ["LIFE_TEMPORAL_ROWS"])  # the A/B tile height (life_kernels.hip)
            want = 0
            for m in sizes:
                ghost = m if kernel == "bit" else K  # byte tiles: compile-time ghost depth K
                nty = -(-4096 // (NW * R - 2 * ghost))
                if kernel == "bit":
                    # 64 pairs per row: two tile columns, the second owning 2 pairs; it runs as bands of 4
                    # lanes, 16 tile rows per workgroup (life_kernels.hip tile_geom / region_items; the dataflow
                    # form's banded items likewise, its no-op padding items not counted)
                    tiles = 2 * nty
                    if os.environ.get("LIFE_FLOW_BANDS" if flow else "LIFE_BANDS", "1") != "0":
                        tiles = nty + -(-nty // 16)
                    per_row = 22 * m  # a pair row: 2 v_alignbit + 2 full adders + 2 rules
                else:  # 128 words per row: three tile columns; drifting frame 12 VALU + pack/unpack 35
                    tiles = 3 * nty
                    per_row = 12 * m + 35
                want += tiles * 64 * NW * R * per_row
            assert n * valu == pytest.approx(want)


# ---------------------------------------------------------------- temporal blocking (bit)
@pytest.mark.parametrize("kernel", ["bit", "byte"])
@pytest.mark.parametrize("nx,ny", [(32, 1), (32, 5), (64, 64), (96, 33), (2048, 100), (1024, 1000), (4096, 48),
                                   (32, 200), (1984, 130), (2016, 7),
                                   # widths not a multiple of 32: the shard wraps its own x-aprons
                                   (33, 9), (63, 64), (500, 500), (1000, 37), (4016, 130), (1985, 3), (2047, 200),
                                   (256, 5000), (100, 3001)])
@pytest.mark.parametrize("flow", [0, 1], ids=["tiles", "flow"])
def test_temporal_single_shard(gpu, oracle, kernel, nx, ny, flow):
    """Blocks at least one lane column wide (bit: a 64-cell pair; byte: 32
    cells) take the temporally blocked kernel (up to K generations per
    launch), narrower ones the one-generation kernel; runs of 1, 7, 8, 9, 20,
    40 and 70 generations.  tiles: one launch per pass; flow: LIFE_OPT_FLOW 1,
    the dataflow tiles (bit) where the shard wraps x in its lane columns (the
    70-generation call: 5 passes of 12, then a 10-generation launch)."""
    temporal = nx >= gpu.TEMPORAL_XAPRON[kernel]
    assert gpu.layout_query(nx, ny, (1, 1), 0, kernel).generations_per_exchange == (
        gpu.TEMPORAL_DEPTH[kernel] if temporal else 1)
    g0 = oracle.fill_random(nx, ny, seed=nx + 3 * ny, density=0.5)
    with gpu.Life(nx, ny, kernel=kernel, small_grid=False, flow=flow) as life:
        life.upload(g0)
        done = 0
        for n in (1, 7, 8, 9, 20, 40, 70):
            life.step(n)
            done += n
            np.testing.assert_array_equal(life.gather(), oracle.life_run(g0, done, threads=4),
                                          err_msg=f"after {done} generations")


@pytest.mark.parametrize("nx,ny,shards,dims", [
    (256, 64, 4, (2, 2)), (512, 80, 8, (4, 2)), (64, 80, 4, (1, 4)), (256, 9, 4, (4, 1)), (64, 20, 2, (2, 1)),
    (96, 32, 6, (3, 2)), (4096, 4096, 4, (2, 2)), (8192, 200, 8, (4, 2)), (2048, 1100, 2, (1, 2)),
    # block widths not a multiple of 32 (remainder rule, straddling columns)
    (500, 500, 2, (2, 1)), (500, 300, 8, (4, 2)), (100, 64, 6, (3, 2)), (1000, 70, 4, (2, 2)), (2047, 90, 2, (1, 2)),
])
@pytest.mark.parametrize("kernel", ["bit", "byte"])
def test_temporal_multi_shard_local(gpu, oracle, kernel, nx, ny, shards, dims):
    """K-deep aprons through the LOCAL transport: whole-word columns, K-row
    blocks of rows, ring tiles first, interior overlapped with the exchange."""
    K = gpu.TEMPORAL_DEPTH[kernel]
    # a partitioned block shorter than K rows, or narrower than one lane column, takes the one-cell path
    wide = dims[0] == 1 or nx // dims[0] >= gpu.TEMPORAL_XAPRON[kernel]
    want = K if wide and (dims[1] == 1 or ny // dims[1] >= K) else 1
    for r in range(shards):
        assert gpu.layout_query(nx, ny, dims, r, kernel).generations_per_exchange == want
    g0 = oracle.fill_random(nx, ny, seed=7 * shards + ny, density=0.45)
    with gpu.Life(nx, ny, shards=shards, kernel=kernel, dims=dims, transport=gpu.XPORT_LOCAL) as life:
        life.upload(g0)
        done = 0
        for n in (1, 8, 13, 16, 30, 40):
            life.step(n)
            done += n
            np.testing.assert_array_equal(life.gather(), oracle.life_run(g0, done, threads=4),
                                          err_msg=f"after {done} generations")


@pytest.mark.parametrize("kernel,rows", [("bit", 16), ("bit", 24), ("byte", 32), ("byte", 48)])
def test_temporal_tile_heights_agree(gpu, oracle, kernel, rows):
    nx, ny = 2048, 333
    g0 = oracle.fill_random(nx, ny, seed=rows, density=0.5)
    gpu.tune_temporal(rows, kernel)
    try:
        with gpu.Life(nx, ny, kernel=kernel, small_grid=False) as life:
            life.upload(g0)
            life.step(40)
            np.testing.assert_array_equal(life.gather(), oracle.life_run(g0, 40, threads=4))
    finally:
        gpu.tune_temporal(gpu.TEMPORAL_ROWS[kernel], kernel)


# ---------------------------------------------------------------- CU-resident small grids
@pytest.mark.parametrize("small", ["lds", True, "vgpr1"], ids=["lds", "vgpr", "vgpr1"])
@pytest.mark.parametrize("kernel", ["bit", "byte"])
@pytest.mark.parametrize("nx,ny,gens", [(500, 500, 300), (1, 1, 5), (33, 2, 17), (31, 31, 40), (1000, 600, 50),
                                        (32768, 19, 9), (64, 3, 100), (97, 1, 12),
                                        # VGPR kernel shapes: strip heights 1..32, 1..64 words per row
                                        (300, 100, 77), (10, 10, 33), (2048, 512, 21), (2047, 480, 19),
                                        (64, 1000, 45), (100, 96, 60), (1, 7, 9), (40, 20, 100),
                                        (1984, 400, 25), (96, 125, 64)])
def test_small_grid_path(gpu, oracle, kernel, nx, ny, gens, small):
    g0 = oracle.fill_random(nx, ny, seed=nx ^ ny, density=0.4)
    with gpu.Life(nx, ny, kernel=kernel, small_grid=small) as life:
        life.upload(g0)
        life.step(gens)
        np.testing.assert_array_equal(life.gather(), oracle.life_run(g0, gens, threads=4))
        life.step(1)
        np.testing.assert_array_equal(life.gather(), oracle.life_run(g0, gens + 1, threads=4))


@pytest.mark.parametrize("kernel", ["bit", "byte"])
@pytest.mark.parametrize("nx,ny,gens,window", [
    (500, 500, 300, None), (500, 500, 77, (4, 32)), (500, 500, 40, (1, 3)),   # p46gun_big's shape
    (64, 1000, 45, None), (2048, 512, 21, None), (1000, 600, 50, None),        # automatic R / K
    (512, 300, 50, None), (481, 97, 33, None), (500, 64, 20, (1, 8)),          # 16-word rows: DPP row rotates
    (2047, 480, 19, (1, 4)), (1984, 400, 25, (2, 8)), (64, 1000, 45, (1, 100)),
    (300, 100, 77, (1, 16)), (1000, 600, 50, (3, 20)), (96, 125, 64, (1, 70)), (10, 10, 33, None)])
def test_small_grid_windowed(gpu, oracle, kernel, nx, ny, gens, window):
    """The VGPR small-grid kernel windowed over ceil(h / own) workgroups
    (K halo rows, K generations per launch; last window partial; shapes it
    does not fit, like 10x10, fall back to the one-workgroup kernel)."""
    g0 = oracle.fill_random(nx, ny, seed=nx ^ ny ^ 5, density=0.4)
    with gpu.Life(nx, ny, kernel=kernel, small_grid="window", window=window) as life:
        life.upload(g0)
        life.step(gens)
        np.testing.assert_array_equal(life.gather(), oracle.life_run(g0, gens, threads=4))
        life.step(1)
        np.testing.assert_array_equal(life.gather(), oracle.life_run(g0, gens + 1, threads=4))


def test_small_grid_window_option_values(gpu, oracle):
    """LIFE_OPT_SMALL_WINDOW: strip heights without a kernel instance and
    K = 0 are rejected; value 0 restores the automatic plan."""
    g0 = oracle.fill_random(500, 500, seed=3, density=0.4)
    with gpu.Life(500, 500, small_grid="window") as life:
        for bad in (7 * 256 + 5, 9 * 256 + 5, 1 * 256 + 0, 5):
            with pytest.raises(gpu.LifeError):
                life.configure(gpu.OPT_SMALL_WINDOW, bad)
        life.configure(gpu.OPT_SMALL_WINDOW, 2 * 256 + 9)
        life.configure(gpu.OPT_SMALL_WINDOW, 0)
        life.upload(g0)
        life.step(61)
        np.testing.assert_array_equal(life.gather(), oracle.life_run(g0, 61, threads=4))


@pytest.mark.parametrize("kernel", ["bit", "byte"])
def test_small_grid_windowed_timing(gpu, oracle, kernel):
    """Kernel stats of the windowed path: one event pair per step call,
    counted as its ceil(gens / K) launches (automatic K = 30 for 16-word
    rows), one grid import + export of HBM bytes per launch."""
    nx, ny, gens = 500, 500, 95
    g0 = oracle.fill_random(nx, ny, seed=46, density=0.4)
    with gpu.Life(nx, ny, kernel=kernel) as life:
        life.upload(g0)
        life.set_timing(True)
        life.step(gens)
        ms, n, b = life.kernel_stats()
        upd, _ = life.kernel_work()
        assert n == 4 and ms > 0  # 30 + 30 + 30 + 5
        assert n * b == pytest.approx(nx * ny * 4 * (0.25 if kernel == "bit" else 2.0))
        assert n * upd == pytest.approx(nx * ny * gens)
        np.testing.assert_array_equal(life.gather(), oracle.life_run(g0, gens, threads=4))


@pytest.mark.parametrize("kernel", ["bit", "byte"])
def test_repeated_gather_is_stable(gpu, oracle, kernel):
    """Host transfers: 12 gathers of a 16 MiB grid into fresh pageable buffers
    all equal the oracle (guards the blocking-copy rule of life_dev_gather)."""
    want = oracle.fill_random(4096, 4096, 1, 0.5)
    with gpu.Life(4096, 4096, kernel=kernel, small_grid=False) as life:
        life.upload(want)
        for _ in range(6):
            np.testing.assert_array_equal(life.gather(), want)
        life.fill_random(1, 0.5)
        for _ in range(6):
            np.testing.assert_array_equal(life.gather(), want)


@pytest.mark.parametrize("kernel", ["bit", "byte"])
def test_step_right_after_async_fill(gpu, oracle, kernel):
    """fill_random is asynchronous on the compute stream; the overlapped
    schedule's interior (second stream) and halo (comm stream) must still see
    the filled grid (life_dev_step's entry fence).  Tall partitioned shards make
    the fill long enough to race without it."""
    nx, ny, gens = 4096, 16384, 33
    with gpu.Life(nx, ny, shards=2, kernel=kernel, dims=(2, 1), transport=gpu.XPORT_LOCAL) as life:
        life.fill_random(9, 0.5)
        life.step(gens)
        got = life.checksum()
    want = oracle.life_run(oracle.fill_random(nx, ny, 9, 0.5), gens, threads=8)
    assert got == oracle.checksum(want)


def test_measure_copy_ceiling(gpu):
    """life_measure_copy (bench's live copy ceiling): a plausible HBM rate
    (MI355X spec 8 TB/s; ~6.3 TB/s measured for a float4 copy)."""
    g = gpu.measure_copy(0, 1 << 30, 3)
    assert 2000.0 < g < 8000.0, g


@pytest.mark.parametrize("kernel", ["byte", "bit"])
@pytest.mark.parametrize("shards,dims,nx,ny", [
    (1, (1, 1), 1000, 37), (1, (1, 1), 7, 5), (1, (1, 1), 4096, 300),
    (6, (3, 2), 1000, 50), (3, (3, 1), 77, 20), (4, (2, 2), 1021, 64), (4, (1, 4), 96, 132), (2, (2, 1), 64, 40),
])
def test_gather_bits(gpu, oracle, kernel, shards, dims, nx, ny):
    """life_dev_gather_bits (the driver's LIFEBITS frame body, packed on the
    device) == np.packbits(gather(), little) -- including blocks whose x
    start is not a multiple of 8, whose edge bytes two shards share."""
    g0 = oracle.fill_random(nx, ny, seed=nx + shards, density=0.5)
    with gpu.Life(nx, ny, shards=shards, kernel=kernel, dims=dims, transport=gpu.XPORT_LOCAL,
                  small_grid=False) as life:
        life.upload(g0)
        life.step(3)
        dense = life.gather()
        np.testing.assert_array_equal(dense, oracle.life_run(g0, 3))
        want = np.packbits(dense, axis=1, bitorder="little")
        out = np.full((ny, (nx + 7) // 8), 0xA5, dtype=np.uint8)  # stale bytes must not survive
        np.testing.assert_array_equal(life.gather_bits(out), want)


@pytest.mark.parametrize("kernel", ["byte", "bit"])
def test_onegen_tunings(gpu, oracle, kernel):
    """Every rows-per-lane x prefetch-depth instance of the one-generation
    stencil (life_tune; depth 18 = a 16-row strip loaded whole, other row
    counts then fall back to 4) on narrow blocks (4 shards of 30-31 columns:
    one-generation layouts for both encodings) with strips cut short by the
    block height -- bit-exact against the oracle."""
    nx, ny = 122, 517
    g0 = oracle.fill_random(nx, ny, seed=77, density=0.45)
    want = oracle.life_run(g0, 5)
    try:
        for rows in (16, 32, 64):
            for depth in (2, 4, 8, 18):
                gpu.tune(rows, depth, kernel=kernel)
                with gpu.Life(nx, ny, shards=4, kernel=kernel, dims=(4, 1), transport=gpu.XPORT_LOCAL,
                              small_grid=False) as life:
                    life.upload(g0)
                    life.step(5)
                    assert life.last_path() == "onegen"
                    np.testing.assert_array_equal(life.gather(), want, err_msg=f"rows={rows} depth={depth}")
    finally:
        gpu.tune(16, 8, kernel="byte")  # the library defaults (life_kernels.hip Tunings)
        gpu.tune(16, 18, kernel="bit")


@pytest.mark.parametrize("pairs,ny,gens,m", [
    (1, 500, 9, 9), (2, 77, 11, 11), (62, 150, 13, 12), (63, 200, 13, 13), (64, 333, 20, 10), (65, 150, 7, 7),
    (126, 100, 25, 12), (127, 190, 10, 10), (128, 64, 32, 32), (189, 90, 12, 6), (190, 40, 31, 31)])
def test_wide_periodic_tile_columns(gpu, oracle, pairs, ny, gens, m):
    """Bit tiles on an x axis that wraps inside the shard, several tile
    columns of 62 pairs: widths around multiples of 62-63 pairs (a last
    column owning 1..30 pairs runs banded, 31..62 as a whole tile), the wrap
    seam between the last column and column 0, m up to 32 -- against the
    oracle.  (63-pair columns with half-pair edges were measured 1.7-2.3 %
    slower than these and dropped, profiles/r03/r5i.)"""
    nx = 64 * pairs
    g0 = oracle.fill_random(nx, ny, seed=pairs * 31 + ny, density=0.45)
    want = oracle.life_run(g0, gens)
    with gpu.Life(nx, ny, kernel="bit", small_grid=False) as life:
        life.configure(gpu.OPT_FLOW, 0)
        life.configure(gpu.OPT_BLOCK_GENS, m)
        life.upload(g0)
        life.step(gens)
        assert life.last_path() == "tiles"
        np.testing.assert_array_equal(life.gather(), want)


# ---------------------------------------------------------------- deep halo (bit, partitioned)
@pytest.mark.parametrize("nx,ny,shards,dims", [
    (512, 300, 4, (2, 2)), (640, 96, 2, (2, 1)), (256, 200, 2, (1, 2)), (1000, 70, 4, (2, 2)),
    (4100, 150, 2, (2, 1)), (2000, 333, 6, (3, 2)), (130, 64, 2, (2, 1)), (64 * 63 * 2, 90, 2, (2, 1))])
@pytest.mark.parametrize("overlap", [True, False], ids=["overlap", "serial"])
def test_deep_halo(gpu, oracle, nx, ny, shards, dims, overlap):
    """LIFE_OPT_DEEP_HALO: one K-deep exchange feeds several passes, the
    passes in between also advance the apron rows / pairs they will read.
    Call patterns that run 1, 2 and 3 passes between exchanges, a pass longer
    than planned (LIFE_OPT_BLOCK_GENS raised mid-run: the exchange is forced
    first), deep off mid-run (the aprons are refilled) -- x-only, y-only and
    2-D partitions, widths with a partial last pair, a 64 * 63-pair block
    (banded / full last tile column) -- against the oracle and against the
    same run with one exchange per pass."""
    g0 = oracle.fill_random(nx, ny, seed=nx + ny + shards, density=0.45)
    calls = [(5, None), (20, None), (7, None), (31, 32), (12, 12), (9, "off"), (33, None), (1, "on"), (24, None)]
    got = {}
    for deep in (1, 0):
        with gpu.Life(nx, ny, shards=shards, kernel="bit", dims=dims, transport=gpu.XPORT_LOCAL,
                      overlap=overlap) as life:
            life.configure(gpu.OPT_DEEP_HALO, deep)
            life.upload(g0)
            done = 0
            for gens, opt in calls:
                if opt == "off":
                    life.configure(gpu.OPT_DEEP_HALO, 0)
                elif opt == "on":
                    life.configure(gpu.OPT_DEEP_HALO, deep)
                elif opt is not None:
                    life.configure(gpu.OPT_BLOCK_GENS, opt)
                life.step(gens)
                done += gens
                if deep:
                    np.testing.assert_array_equal(life.gather(), oracle.life_run(g0, done, threads=4),
                                                  err_msg=f"after {done} generations")
            got[deep] = life.gather()
    np.testing.assert_array_equal(got[1], got[0])


@pytest.mark.parametrize("rccl", [None, "rank"], ids=["local", "rccl"])
def test_deep_halo_exchange_count(gpu, oracle, rccl):
    """The exchange count the deep halo buys: on the loopback (the shard its
    own neighbour, RCCL or LOCAL), a 5-generation call, then a 20-generation
    call (2 passes of 10, the driver's shape) records ONE overlapped block --
    one exchange for 25 generations -- where the per-pass schedule records 3."""
    nx, ny = 4096, 1024
    g0 = oracle.fill_random(nx, ny, seed=23, density=0.5)
    for deep, blocks in ((1, 1), (0, 3)):
        life = (gpu.Life.for_rank(nx, ny, 0, 1, gpu.unique_id(), 0, kernel="bit") if rccl
                else gpu.Life(nx, ny, kernel="bit"))
        with life:
            life.upload(g0)
            life.configure(gpu.OPT_LOOPBACK, 1)
            life.configure(gpu.OPT_DEEP_HALO, deep)
            life.set_timing(True)
            life.step(5)
            life.step(20)
            assert life.phase_stats()["blocks"] == blocks
            np.testing.assert_array_equal(life.gather(), oracle.life_run(g0, 25, threads=4))





_TIMING_OFF = r"""
import sys
sys.path.insert(0, {pkg!r})
import life_mi355x as lm
for flow in (0, 1):
    with lm.Life(4096, 4096, kernel="bit", small_grid=False, flow=flow) as life:
        life.fill_random(1)
        life.set_timing(True)
        life.step(72)
        path = life.last_path()
        assert path == ("flow" if flow else "tiles"), path
        ms, n, b = life.kernel_stats()
        upd, valu = life.kernel_work()
        assert (n, b, upd, valu) == (0, 0.0, 0.0, 0.0), (path, n, b, upd, valu)
print("TIMING_OFF_OK", flush=True)
"""


def test_timing_mode_off_books_nothing(gpu):
    """under LIFE_TIMING_MODE=3 no launch is timed, so no
    work may be booked either -- the tiles and the dataflow passes alike --
    or bytes / updates per launch come out of a count of zero launches."""
    import subprocess
    import sys

    from conftest import ROOT

    env = dict(os.environ, LIFE_TIMING_MODE="3")
    out = subprocess.run([sys.executable, "-c", _TIMING_OFF.format(pkg=os.path.join(ROOT, "mpi-and-open-mp_amd"))],
                         env=env, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0 and "TIMING_OFF_OK" in out.stdout, out.stdout + out.stderr
