"""life_mi355x -- Python binding of the MI355X Game-of-Life C ABI.

Mirrors the reference's per-rank interface (6-cartesian/life_cart.c:39-49):

=====================  ==============================================
reference              here
=====================  ==============================================
life_init (loader)     :func:`load_cfg` (cfg.py) + :class:`Life`
life_step              :meth:`Life.step`  (HIP kernels)
life_exchange          part of :meth:`Life.step` (RCCL / local halo)
life_collect           :meth:`Life.gather` (device-side gather)
life_save_vtk          :func:`save_vtk` (cfg.py)
decomposition          :func:`decomposition`
MPI_Dims_create        :func:`dims_create`
life_free              :meth:`Life.close`
=====================  ==============================================

The compute path is ``liblife_mi355x.so`` only: there is no CPU fallback.
Importing works without a GPU (host-only helpers such as
:func:`halo_plan` run anywhere); device calls raise :class:`LifeError` when
no HIP device is present.
"""
from __future__ import annotations

import ctypes
import importlib.abc
import os
import sys

import numpy as np

from .cfg import bits_bytes, load_bits, load_cfg, save_vtk, vtk_bytes, vtk_header  # noqa: F401

HERE = os.path.dirname(os.path.abspath(__file__))
# LIFE_MI355X_LIB: load another build of the same library (experiments only)
LIB_PATH = os.environ.get("LIFE_MI355X_LIB") or os.path.join(HERE, "liblife_mi355x.so")

KERNEL_BYTE = 0
KERNEL_BIT = 1
KERNELS = {"byte": KERNEL_BYTE, "bit": KERNEL_BIT}
XPORT_AUTO, XPORT_RCCL, XPORT_LOCAL = 0, 1, 2
HALO_SEND, HALO_RECV, HALO_FILL = 0, 1, 2
HALO_COLUMN, HALO_ROW, HALO_CORNER = 0, 1, 2
OPT_SMALL_GRID, OPT_OVERLAP, OPT_SMALL_WINDOW, OPT_BLOCK_GENS, OPT_LOOPBACK, OPT_FLOW = 1, 2, 4, 5, 6, 7
OPT_FLOW_CHUNK = 8
OPT_DEEP_HALO = 9
# LIFE_TEMPORAL_DEPTH(_BYTE): generations per halo exchange of the temporal layouts
TEMPORAL_DEPTH = {"bit": 32, "byte": 32}
BLOCK_GENS = {"bit": 12, "byte": 32}  # tiles: default generations per launch at most (LIFE_OPT_BLOCK_GENS)
TEMPORAL_ROWS = {"bit": 24, "byte": 48}  # default register rows per wave (bit: 64-cell pair rows)
TILE_WAVES = {"bit": 8, "byte": 8}  # waves per tile workgroup (window = waves x rows)
TEMPORAL_XAPRON = {"bit": 64, "byte": 32}  # x-apron of the temporal layouts: one lane column

# Every symbol include/life_mi355x.h declares (checked by tests/test_abi.py).
ABI_SYMBOLS = (
    "life_decomposition", "life_dims_create", "life_dims_choose", "life_halo_plan", "life_layout_query",
    "life_strerror", "life_last_error", "life_dev_create", "life_dev_create_ex",
    "life_get_unique_id", "life_dev_create_rank", "life_dev_upload", "life_dev_fill_random",
    "life_dev_step", "life_dev_gather", "life_dev_live_count", "life_dev_sync",
    "life_dev_layout", "life_dev_world", "life_dev_set_timing", "life_dev_kernel_stats",
    "life_tune", "life_tune_temporal", "life_dev_configure", "life_dev_kernel_work", "life_dev_checksum",
    "life_dev_gather_vtk", "life_dev_gather_bits", "life_dev_destroy", "life_measure_copy", "life_dev_phase_stats",
    "life_dev_barrier", "life_device_count", "life_dev_last_path", "life_dev_call_stats",
    "life_dev_strerror", "life_dev_shard_info",
)
PATHS = {0: "none", 1: "onegen", 2: "tiles", 3: "flow", 5: "small"}


class LifeError(RuntimeError):
    def __init__(self, rc: int, what: str):
        lib = _lib()
        detail = lib.life_last_error().decode(errors="replace")
        super().__init__(f"{what}: {lib.life_strerror(rc).decode()} ({rc}){': ' + detail if detail else ''}")
        self.rc = rc


class HaloOp(ctypes.Structure):
    _fields_ = [("phase", ctypes.c_int32), ("kind", ctypes.c_int32), ("peer", ctypes.c_int32),
                ("what", ctypes.c_int32), ("index", ctypes.c_int64), ("first", ctypes.c_int64),
                ("count", ctypes.c_int64), ("width", ctypes.c_int64)]

    def as_tuple(self):
        return (self.phase, self.kind, self.peer, self.what, self.index, self.first, self.count, self.width)


class Layout(ctypes.Structure):
    _fields_ = [("w", ctypes.c_int64), ("h", ctypes.c_int64), ("x0", ctypes.c_int64),
                ("y0", ctypes.c_int64), ("pitch", ctypes.c_int64), ("xoff", ctypes.c_int64),
                ("rows", ctypes.c_int64), ("units", ctypes.c_int64), ("xapron", ctypes.c_int64),
                ("yapron", ctypes.c_int64), ("kernel", ctypes.c_int32), ("coords", ctypes.c_int32 * 2),
                ("generations_per_exchange", ctypes.c_int32), ("reserved", ctypes.c_int32)]


_LIB = None


class _TorchAfterLibraryGuard(importlib.abc.MetaPathFinder):
    """Refuses `import torch` once liblife_mi355x.so is loaded:
    the library binds /opt/rocm's libamdhip64.so.7; torch links its bundled HIP
    runtime by the unversioned name, so importing it afterwards maps a SECOND
    runtime into the process and it dies with a double free at exit.  With
    torch imported first, the library binds torch's runtime and all is well."""

    MESSAGE = ("life_mi355x: liblife_mi355x.so is already loaded with /opt/rocm's HIP runtime; importing torch now "
               "would map torch's bundled HIP runtime as a second copy (the process aborts with a double free at "
               "exit).  Import torch before the first life_mi355x device call, or not at all.")

    def find_spec(self, name, path, target=None):
        if name == "torch" or name.startswith("torch."):
            raise ImportError(self.MESSAGE)
        return None


def _lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is not built: run `make -C mpi-and-open-mp_amd` "
                              "or __graft_entry__.build()")
        if "torch" not in sys.modules and not any(isinstance(f, _TorchAfterLibraryGuard) for f in sys.meta_path):
            sys.meta_path.insert(0, _TorchAfterLibraryGuard())
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        i64, i32, vp = ctypes.c_int64, ctypes.c_int, ctypes.c_void_p
        P = ctypes.POINTER
        L.life_decomposition.argtypes = [i64, i32, i32, P(i64), P(i64)]
        L.life_decomposition.restype = None
        L.life_dims_create.argtypes = [i32, P(ctypes.c_int)]
        L.life_dims_create.restype = None
        L.life_dims_choose.argtypes = [i64, i64, i32, i32, P(ctypes.c_int)]
        L.life_halo_plan.argtypes = [i64, i64, i32, i32, i32, i32, P(HaloOp), i32]
        L.life_layout_query.argtypes = [i64, i64, i32, i32, i32, i32, P(Layout)]
        L.life_strerror.argtypes = [i32]
        L.life_strerror.restype = ctypes.c_char_p
        L.life_last_error.restype = ctypes.c_char_p
        L.life_dev_create.argtypes = [i64, i64, i32, i32, P(vp)]
        L.life_dev_create_ex.argtypes = [i64, i64, i32, i32, i32, i32, i32, P(vp)]
        L.life_get_unique_id.argtypes = [ctypes.c_char_p]
        L.life_dev_create_rank.argtypes = [i64, i64, i32, i32, i32, i32, i32, ctypes.c_char_p, i32, P(vp)]
        L.life_dev_upload.argtypes = [vp, P(ctypes.c_uint8)]
        L.life_dev_fill_random.argtypes = [vp, ctypes.c_uint64, ctypes.c_uint32]
        L.life_dev_step.argtypes = [vp, i64]
        L.life_dev_gather.argtypes = [vp, P(ctypes.c_uint8)]
        L.life_dev_gather_vtk.argtypes = [vp, ctypes.c_char_p]
        L.life_dev_gather_bits.argtypes = [vp, ctypes.POINTER(ctypes.c_uint8)]
        L.life_dev_live_count.argtypes = [vp]
        L.life_dev_live_count.restype = i64
        L.life_dev_sync.argtypes = [vp]
        L.life_dev_barrier.argtypes = [vp]
        L.life_device_count.argtypes = []
        L.life_dev_last_path.argtypes = [vp]
        L.life_dev_checksum.argtypes = [vp, P(ctypes.c_uint64)]
        L.life_dev_layout.argtypes = [vp, i32, P(Layout)]
        L.life_dev_world.argtypes = [vp] + [P(ctypes.c_int)] * 5
        L.life_dev_set_timing.argtypes = [vp, i32]
        L.life_dev_configure.argtypes = [vp, i32, i32]
        L.life_dev_kernel_stats.argtypes = [vp, P(ctypes.c_double), P(i64), P(ctypes.c_double)]
        L.life_dev_kernel_work.argtypes = [vp, P(ctypes.c_double), P(ctypes.c_double)]
        L.life_dev_phase_stats.argtypes = [vp] + [P(ctypes.c_double)] * 4 + [P(i64)]
        if hasattr(L, "life_dev_call_stats"):  # absent from pre-round-4 builds (LIFE_MI355X_LIB A/B runs)
            L.life_dev_call_stats.argtypes = [vp, P(ctypes.c_double), P(ctypes.c_double), P(i64), P(ctypes.c_double)]
        if hasattr(L, "life_dev_shard_info"):  # absent from pre-round-6 builds (LIFE_MI355X_LIB A/B runs)
            L.life_dev_shard_info.argtypes = [vp, i32, P(ctypes.c_int), ctypes.c_char_p, P(ctypes.c_int)]
        L.life_tune.argtypes = [i32, i32, i32]
        L.life_tune_temporal.argtypes = [i32, i32]
        L.life_measure_copy.argtypes = [i32, i64, i32, P(ctypes.c_double)]
        L.life_dev_destroy.argtypes = [vp]
        L.life_dev_destroy.restype = None
        _LIB = L
    return _LIB


# Test hook: a byte value that fresh gather destinations are filled with
# before the device copy (None: np.empty).  tests/conftest.py sets 0xA5, so a
# copy that did not land shows up as poison instead of as a plausible grid.
GATHER_FILL = None


def _host_buffer(shape) -> np.ndarray:
    if GATHER_FILL is None:
        return np.empty(shape, dtype=np.uint8)
    return np.full(shape, GATHER_FILL, dtype=np.uint8)


def _check(rc: int, what: str) -> int:
    if rc < 0:
        raise LifeError(rc, what)
    return rc


def kernel_id(kernel) -> int:
    if isinstance(kernel, str):
        return KERNELS[kernel]
    return int(kernel)


# ---------------------------------------------------------------- host only
def decomposition(n: int, p: int, k: int):
    """life_cart.c:217-223 -> (start, stop)."""
    s, e = ctypes.c_int64(), ctypes.c_int64()
    _lib().life_decomposition(n, p, k, ctypes.byref(s), ctypes.byref(e))
    return s.value, e.value


def dims_create(n: int):
    """MPI_Dims_create(n, 2, {0,0}) (life_cart.c:117-118)."""
    d = (ctypes.c_int * 2)()
    _lib().life_dims_create(n, d)
    return d[0], d[1]


PARTITIONS = {"cart": 0, "rows": 1, "cols": 2, "auto": 3}  # LIFE_PARTITION_*


def dims_choose(nx: int, ny: int, n: int, policy="auto"):
    """Partition shape for n shards (life_dims_choose): "cart" =
    MPI_Dims_create, "rows" = {1, n} strips, "cols" = {n, 1}, "auto"."""
    d = (ctypes.c_int * 2)()
    pol = PARTITIONS[policy] if isinstance(policy, str) else int(policy)
    _check(_lib().life_dims_choose(nx, ny, n, pol, d), "life_dims_choose")
    return d[0], d[1]


def halo_plan(nx: int, ny: int, dims, rank: int, kernel="byte"):
    """The per-exchange halo ops of shard `rank` (see life_halo_plan)."""
    ops = (HaloOp * 16)()
    n = _check(_lib().life_halo_plan(nx, ny, dims[0], dims[1], rank, kernel_id(kernel), ops, 16),
               "life_halo_plan")
    return [ops[i].as_tuple() for i in range(n)]


def layout_query(nx: int, ny: int, dims, rank: int, kernel="byte") -> Layout:
    L = Layout()
    _check(_lib().life_layout_query(nx, ny, dims[0], dims[1], rank, kernel_id(kernel), ctypes.byref(L)),
           "life_layout_query")
    return L


def density_to_thr(density: float) -> int:
    return min(int(density * 2.0**32), 0xFFFFFFFF)


def tune_temporal(rows: int = 0, kernel=-1) -> None:
    """Temporal tile height: register rows per wave of one encoding (bit:
    16/24 pair rows; byte: 32/48 word rows), or of both
    (kernel -1: each takes the value if valid for it)."""
    _check(_lib().life_tune_temporal(kernel_id(kernel), rows), "life_tune_temporal")


def tune(rows: int = 0, depth: int = 0, kernel=-1) -> None:
    """Stencil rows-per-lane / prefetch depth for this process (life_tune)."""
    _check(_lib().life_tune(kernel_id(kernel), rows, depth), "life_tune")


def measure_copy(device: int = 0, nbytes: int = 2 << 30, reps: int = 5) -> float:
    """Measured HBM copy ceiling in GB/s (read + write bytes / best time)."""
    g = ctypes.c_double()
    _check(_lib().life_measure_copy(device, nbytes, reps, ctypes.byref(g)), "life_measure_copy")
    return g.value


def unique_id() -> bytes:
    buf = ctypes.create_string_buffer(128)
    _check(_lib().life_get_unique_id(buf), "life_get_unique_id")
    return buf.raw


# ---------------------------------------------------------------- device
class Life:
    """A periodic nx x ny Game of Life resident in MI355X HBM.

    ``Life(nx, ny, shards=1, kernel="bit")`` drives ``shards`` Cartesian
    blocks from this process (one per GPU, or several logical shards on one
    GPU with the LOCAL transport).  :meth:`for_rank` is the
    one-process-per-GPU form (torchrun), with RCCL between ranks.
    """

    def __init__(self, nx: int, ny: int, shards: int = 1, kernel="bit", dims=(0, 0),
                 transport: int = XPORT_AUTO, small_grid: bool = True, overlap: bool = True, flow=None,
                 window=None, _handle=None):
        self.nx, self.ny = int(nx), int(ny)
        self.kernel = kernel_id(kernel)
        self._h = ctypes.c_void_p()
        if _handle is not None:
            self._h = _handle
        else:
            _check(_lib().life_dev_create_ex(self.nx, self.ny, shards, dims[0], dims[1], self.kernel,
                                             transport, ctypes.byref(self._h)), "life_dev_create")
        # small_grid: True/"auto" (VGPR kernel when the shape allows, else LDS),
        # "lds" (LDS kernel only), "window" (the VGPR kernel windowed over
        # several CUs where the shape allows, else as True; True windows only
        # shapes whose one-workgroup strips would be >= 4 rows tall), "vgpr1"
        # (as True, never windowed), False (the streaming kernels);
        # window=(R, K): the windowed kernel's strip height and halo rows
        mode = {True: 1, "auto": 1, "lds": 2, "window": 3, "vgpr1": 4, False: 0}[small_grid]
        if mode != 1:
            self.configure(OPT_SMALL_GRID, mode)
        if window is not None:
            self.configure(OPT_SMALL_WINDOW, int(window[0]) * 256 + int(window[1]))
        if not overlap:
            self.configure(OPT_OVERLAP, 0)
        # flow: None (library default 3: the dataflow tiles where a pass is
        # only a few rounds of workgroups), or a LIFE_OPT_FLOW value (0: one
        # launch per pass)
        if flow is not None:
            self.configure(OPT_FLOW, int(flow))

    def configure(self, option: int, value: int) -> None:
        _check(_lib().life_dev_configure(self._h, option, value), "configure")

    @classmethod
    def for_rank(cls, nx, ny, rank, world, uid: bytes, device: int, kernel="bit", dims=(0, 0)):
        h = ctypes.c_void_p()
        _check(_lib().life_dev_create_rank(nx, ny, kernel_id(kernel), rank, world, dims[0], dims[1],
                                           uid, device, ctypes.byref(h)), "life_dev_create_rank")
        return cls(nx, ny, kernel=kernel, _handle=h)

    # life_init's cell loading (life_cart.c:104-109)
    def upload(self, grid: np.ndarray) -> None:
        g = np.ascontiguousarray(grid, dtype=np.uint8)
        if g.shape != (self.ny, self.nx):
            raise ValueError(f"grid shape {g.shape} != ({self.ny}, {self.nx})")
        _check(_lib().life_dev_upload(self._h, g.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))), "upload")

    def fill_random(self, seed: int, density: float = 0.5) -> None:
        _check(_lib().life_dev_fill_random(self._h, seed, density_to_thr(density)), "fill_random")

    def step(self, generations: int = 1) -> None:
        _check(_lib().life_dev_step(self._h, generations), "step")

    def gather(self, out: np.ndarray | None = None) -> np.ndarray:
        if out is None:
            out = _host_buffer((self.ny, self.nx))
        _check(_lib().life_dev_gather(self._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))), "gather")
        return out

    def gather_vtk(self) -> bytes:
        """life_dev_gather_vtk: the whole VTK file of the current grid, with
        the cell text formatted on the device (== save_vtk of gather())."""
        body = ctypes.create_string_buffer(2 * self.nx * self.ny)
        _check(_lib().life_dev_gather_vtk(self._h, body), "gather_vtk")
        return vtk_header(self.nx, self.ny) + body.raw

    def gather_bits(self, out: np.ndarray | None = None) -> np.ndarray:
        """life_dev_gather_bits: packed rows (ny x ceil(nx/8) bytes, cell x at
        bit x & 7 of byte x >> 3; == np.packbits(gather(), axis=1,
        bitorder="little")), packed on the device."""
        if out is None:
            out = _host_buffer((self.ny, (self.nx + 7) // 8))
        if out.shape != (self.ny, (self.nx + 7) // 8) or out.dtype != np.uint8 or not out.flags.c_contiguous:
            raise ValueError("gather_bits: out must be a C-contiguous uint8 (ny, ceil(nx/8)) array")
        _check(_lib().life_dev_gather_bits(self._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))), "gather_bits")
        return out

    def live_count(self) -> int:
        return _check(_lib().life_dev_live_count(self._h), "live_count")

    def checksum(self) -> int:
        """life_dev_checksum: encoding- and partition-independent grid hash."""
        v = ctypes.c_uint64()
        _check(_lib().life_dev_checksum(self._h, ctypes.byref(v)), "checksum")
        return v.value

    def sync(self) -> None:
        _check(_lib().life_dev_sync(self._h), "sync")

    def barrier(self) -> None:
        """life_dev_barrier: sync, then (rank mode) an all-reduce every rank joins."""
        _check(_lib().life_dev_barrier(self._h), "barrier")

    def layout(self, local_shard: int = 0) -> Layout:
        L = Layout()
        _check(_lib().life_dev_layout(self._h, local_shard, ctypes.byref(L)), "layout")
        return L

    def world(self):
        v = [ctypes.c_int() for _ in range(5)]
        _check(_lib().life_dev_world(self._h, *[ctypes.byref(x) for x in v]), "world")
        return dict(zip(("world", "dims0", "dims1", "nlocal", "transport"), (x.value for x in v)))

    def shard_info(self, local_shard: int = 0):
        """life_dev_shard_info: {"device", "pci_bus_id", "rccl_nranks"} of a
        local shard (rccl_nranks 0: no communicator); None from builds that
        predate it."""
        if not hasattr(_lib(), "life_dev_shard_info"):
            return None
        dev, n = ctypes.c_int(), ctypes.c_int()
        bus = ctypes.create_string_buffer(64)
        _check(_lib().life_dev_shard_info(self._h, local_shard, ctypes.byref(dev), bus, ctypes.byref(n)),
               "shard_info")
        return {"device": dev.value, "pci_bus_id": bus.value.decode(errors="replace"), "rccl_nranks": n.value}

    def set_timing(self, on) -> None:
        """life_dev_set_timing: False off, True launch timing + phase events,
        2 launch timing only (no event packets inside a partitioned step)."""
        _check(_lib().life_dev_set_timing(self._h, int(on)), "set_timing")

    def last_path(self) -> str:
        """Kernel family of the last step call (life_dev_last_path)."""
        return PATHS[_check(_lib().life_dev_last_path(self._h), "last_path")]

    def flow_active(self) -> bool:
        return self.last_path() == "flow"

    def kernel_stats(self):
        ms, n, b = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
        _check(_lib().life_dev_kernel_stats(self._h, ctypes.byref(ms), ctypes.byref(n), ctypes.byref(b)),
               "kernel_stats")
        return ms.value, n.value, b.value

    def kernel_work(self):
        """(cell-updates, VALU lane-ops) per timed launch (life_dev_kernel_work)."""
        u, v = ctypes.c_double(), ctypes.c_double()
        _check(_lib().life_dev_kernel_work(self._h, ctypes.byref(u), ctypes.byref(v)), "kernel_work")
        return u.value, v.value

    def phase_stats(self):
        """Mean ms per overlapped block of the ring, interior, halo exchange
        and whole block, and the number of blocks (life_dev_phase_stats)."""
        v = [ctypes.c_double() for _ in range(4)]
        n = ctypes.c_int64()
        _check(_lib().life_dev_phase_stats(self._h, *[ctypes.byref(x) for x in v], ctypes.byref(n)), "phase_stats")
        return dict(zip(("ring_ms", "interior_ms", "halo_ms", "block_ms"), (x.value for x in v)), blocks=n.value)

    def call_stats(self):
        """Where the last step call's time went (life_dev_call_stats, timing
        on): host enqueue ms (whole call, longest pass), passes, device span
        ms (first work start to last work end, max over local shards)."""
        h, pm, sp = ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        n = ctypes.c_int64()
        if not hasattr(_lib(), "life_dev_call_stats"):
            return {"host_enqueue_ms": 0.0, "pass_enqueue_max_ms": 0.0, "passes": 0, "device_span_ms": 0.0}
        _check(_lib().life_dev_call_stats(self._h, ctypes.byref(h), ctypes.byref(pm), ctypes.byref(n),
                                          ctypes.byref(sp)), "call_stats")
        return {"host_enqueue_ms": h.value, "pass_enqueue_max_ms": pm.value, "passes": n.value,
                "device_span_ms": sp.value}

    def close(self) -> None:
        if self._h:
            _lib().life_dev_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
