"""The multi-GPU halo data path executed on one GPU (LIFE_OPT_LOOPBACK).

A single shard configured as a periodic Cartesian partition of itself: both
axes' aprons come from halo messages the shard sends to itself (two sends
and two receives to ONE peer per phase, matched in order -- the dims = 2 case
of life_cart.c:225-279), with the boundary ring, the halo on the comm stream
and the interior on the second compute stream overlapped as on N GPUs.  Over
a rank-mode device (life_dev_create_rank, world 1, a unique id) the messages
are RCCL ncclSend/ncclRecv: the RCCL branch of the exchange, its message
sizes, group semantics and pack/unpack run here on the one-GPU box.  The
bar is bit-exact against the oracle (3-life/life2d.c:104-130 restated) and
against the same grid stepped without the loopback.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# nx, ny, generations: temporal bit/byte layouts with whole and partial
# words, several halo periods and a partial one; one-generation layouts
# (w < 32); a grid exactly one halo deep
CASES = [(256, 130, 45), (257, 131, 37), (512, 300, 70), (300, 64, 33), (31, 100, 9), (64, 32, 40), (1000, 37, 5)]


def _make(gpu, nx, ny, kernel, rccl):
    if rccl == "rank":  # one-process-per-GPU set-up: ncclCommInitRank at world 1
        return gpu.Life.for_rank(nx, ny, 0, 1, gpu.unique_id(), 0, kernel=kernel)
    if rccl == "initall":  # single-process multi-device set-up: ncclCommInitAll over one device
        return gpu.Life(nx, ny, kernel=kernel, transport=gpu.XPORT_RCCL)
    return gpu.Life(nx, ny, kernel=kernel)


@pytest.mark.parametrize("rccl", [None, "rank", "initall"], ids=["local", "rccl", "rccl_initall"])
@pytest.mark.parametrize("kernel", ["bit", "byte"])
@pytest.mark.parametrize("nx,ny,gens", CASES)
def test_loopback_parity(gpu, oracle, nx, ny, gens, kernel, rccl):
    g0 = oracle.fill_random(nx, ny, seed=11, density=0.4)
    want = oracle.life_run(g0, gens)
    with _make(gpu, nx, ny, kernel, rccl) as life:
        if life.layout().h < life.layout().generations_per_exchange:
            with pytest.raises(RuntimeError):
                life.configure(gpu.OPT_LOOPBACK, 1)
            return
        life.upload(g0)
        life.configure(gpu.OPT_LOOPBACK, 1)
        split = gens // 3
        life.step(split)  # two calls: the schedule is re-entered mid-run
        life.step(gens - split)
        np.testing.assert_array_equal(life.gather(), want)
        assert life.live_count() == int(want.sum())


@pytest.mark.parametrize("kernel", ["bit", "byte"])
def test_loopback_no_overlap_and_toggle(gpu, oracle, kernel):
    """Serial schedule (overlap off), and loopback switched on and off
    between step calls: the aprons are refilled from the shard each time."""
    nx, ny = 320, 200
    g0 = oracle.fill_random(nx, ny, seed=3, density=0.5)
    with gpu.Life(nx, ny, kernel=kernel, overlap=False) as life:
        life.upload(g0)
        life.configure(gpu.OPT_LOOPBACK, 1)
        life.step(21)
        life.configure(gpu.OPT_LOOPBACK, 0)
        life.step(13)
        life.configure(gpu.OPT_LOOPBACK, 1)
        life.step(40)
        np.testing.assert_array_equal(life.gather(), oracle.life_run(g0, 74))


@pytest.mark.parametrize("rccl", [None, "rank"], ids=["local", "rccl"])
def test_loopback_timing_modes(gpu, oracle, rccl):
    """set_timing(True) records the overlapped schedule's phase events,
    set_timing(2) times the launches only: no phase blocks, the tile launches
    still counted and timed; set_timing(3) (bench.py's timed call of a
    multi-stream step) records the call's span only: no launches booked, a
    device span; the same cells throughout."""
    nx, ny, gens = 16384, 1024, 96  # 4 x 3 interior tiles: the interior is its own launch
    g0 = oracle.fill_random(nx, ny, seed=17, density=0.5)
    with _make(gpu, nx, ny, "bit", rccl) as life:
        life.upload(g0)
        life.configure(gpu.OPT_LOOPBACK, 1)
        life.set_timing(True)
        life.step(24)
        # 12 + 12: the deep halo (LIFE_OPT_DEEP_HALO) skips the exchange after
        # the first pass (its successor still fits the K = 32 apron): one
        # overlapped block
        assert life.phase_stats()["blocks"] == 1
        ms1, n1, _ = life.kernel_stats()
        assert n1 == 2 and ms1 > 0  # the interior launches
        life.set_timing(2)
        life.step(40)
        ph = life.phase_stats()
        assert ph["blocks"] == 0 and ph["block_ms"] == 0.0
        ms2, n2, _ = life.kernel_stats()
        assert n2 == 4 and ms2 > 0  # 10 x 4 generations
        np.testing.assert_array_equal(life.gather(), oracle.life_run(g0, 64, threads=4))
        life.set_timing(3)
        life.step(gens - 64)
        assert life.phase_stats()["blocks"] == 0
        assert life.kernel_stats()[1] == 0
        assert life.call_stats()["device_span_ms"] > 0
        np.testing.assert_array_equal(life.gather(), oracle.life_run(g0, gens, threads=4))


def test_loopback_rejected_for_partitioned(gpu):
    with gpu.Life(512, 512, shards=2, kernel="bit", transport=gpu.XPORT_LOCAL) as life:
        with pytest.raises(RuntimeError):
            life.configure(gpu.OPT_LOOPBACK, 1)


@pytest.mark.parametrize("kernel", ["bit", "byte"])
@pytest.mark.parametrize("rccl", ["rank", "initall"])
def test_loopback_rccl_8192(gpu, kernel, rccl):
    """8192^2 over RCCL loopback == the wrapped single shard (census checksum
    and live count after several halo periods and a partial one), through
    either communicator set-up."""
    n = 8192
    with gpu.Life(n, n, kernel=kernel) as ref:
        ref.fill_random(9, 0.5)
        K = ref.layout().generations_per_exchange
        gens = 3 * K + 5
        ref.step(gens)
        want = (ref.checksum(), ref.live_count())
    with _make(gpu, n, n, kernel, rccl) as life:
        life.fill_random(9, 0.5)
        life.configure(gpu.OPT_LOOPBACK, 1)
        life.step(gens)
        assert (life.checksum(), life.live_count()) == want


def test_initall_world(gpu):
    """The single-process RCCL device reports its transport (what bench.py
    --gpus N takes with N real devices)."""
    with gpu.Life(256, 256, kernel="bit", transport=gpu.XPORT_RCCL) as life:
        w = life.world()
        assert (w["world"], w["nlocal"], w["transport"]) == (1, 1, gpu.XPORT_RCCL)


@pytest.mark.parametrize("kernel", ["bit", "byte"])
def test_loopback_initall_gather_and_frames(gpu, oracle, kernel):
    """Gather, VTK and LIFEBITS frames of an RCCL-loopback device after a
    partial halo period equal the oracle's."""
    nx, ny, gens = 640, 96, 45
    g0 = oracle.fill_random(nx, ny, seed=5, density=0.5)
    want = oracle.life_run(g0, gens)
    with gpu.Life(nx, ny, kernel=kernel, transport=gpu.XPORT_RCCL) as life:
        life.upload(g0)
        life.configure(gpu.OPT_LOOPBACK, 1)
        life.step(gens)
        np.testing.assert_array_equal(life.gather(), want)
        np.testing.assert_array_equal(life.gather_bits(), np.packbits(want, axis=1, bitorder="little"))
        assert life.gather_vtk() == gpu.vtk_bytes(want)


@pytest.mark.parametrize("rccl", [None, "rank"], ids=["local", "rccl"])
@pytest.mark.parametrize("kernel", ["bit", "byte"])
@pytest.mark.parametrize("axes", [2, 3], ids=["x_only", "y_only"])
@pytest.mark.parametrize("nx,ny,gens", [(512, 300, 70), (257, 131, 37), (4096, 400, 45)])
def test_loopback_one_axis(gpu, oracle, nx, ny, gens, kernel, rccl, axes):
    """LIFE_OPT_LOOPBACK 2 / 3: only x (as N = 2's {2, 1} blocks) or only y
    goes through the transport, the other axis wraps in the stencil (or its
    own apron copy for a width that is not a whole number of lane columns)."""
    g0 = oracle.fill_random(nx, ny, seed=23, density=0.45)
    want = oracle.life_run(g0, gens)
    with _make(gpu, nx, ny, kernel, rccl) as life:
        life.upload(g0)
        life.configure(gpu.OPT_LOOPBACK, axes)
        split = gens // 3
        life.step(split)
        life.step(gens - split)
        np.testing.assert_array_equal(life.gather(), want)


_INTERIOR_TAIL = r"""
import sys
sys.path.insert(0, {pkg!r})
import life_mi355x as lm
for nx, ny in ((16384, 32768), (32768, 16384)):
    with lm.Life(nx, ny, kernel="bit", flow=0) as life:
        life.fill_random(9, 0.5)
        life.step(77)
        want = (life.checksum(), life.live_count())
    for axes in (1, 2):
        with lm.Life.for_rank(nx, ny, 0, 1, lm.unique_id(), 0, kernel="bit") as life:
            life.fill_random(9, 0.5)
            life.configure(lm.OPT_LOOPBACK, axes)
            life.step(30)
            life.step(47)
            got = (life.checksum(), life.live_count())
            assert got == want, (nx, ny, axes, got, want)
print("INTERIOR_TAIL_OK", flush=True)
"""


@pytest.mark.parametrize("tail", ["0", "1"], ids=["default", "interior_tail"])
def test_exchange_pass_interior_tail(gpu, tail):
    """Round 6: with LIFE_INTERIOR_TAIL=1 the exchange pass's interior launch
    takes the banded half-height tail too, planned with the ring's tiles
    (dispatched just before it on the other stream) counted as holding their
    slots -- configs[3]'s N = 8 block: 567 interior tiles beside 247 ring
    tiles; off by default.  Both settings (the knob is read
    once per process, hence the subprocess): the RCCL-loopback run (several
    exchange blocks, both axes or x only) against the same grid run
    unpartitioned (itself pinned to the oracle by test_gpu_fullsize's
    banded-tail band checks), by census."""
    import os
    import subprocess
    import sys

    from conftest import ROOT

    env = dict(os.environ, LIFE_INTERIOR_TAIL=tail)
    out = subprocess.run([sys.executable, "-c", _INTERIOR_TAIL.format(pkg=os.path.join(ROOT, "mpi-and-open-mp_amd"))],
                         env=env, capture_output=True, text=True, timeout=110)
    assert out.returncode == 0 and "INTERIOR_TAIL_OK" in out.stdout, out.stdout + out.stderr
