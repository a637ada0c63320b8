#!/usr/bin/env python3
"""Benchmark of the MI355X Game-of-Life hot path (one JSON line on rank 0).

A "step" is one generation (halo exchange + B3/S23 update) over the whole
grid.  Default workload (BASELINE.json configs[4], weak scaling): a random
50%-density 65536 x 65536 block per GPU, global grid
(65536*dims0) x (65536*dims1); N = 1 is the 65536^2 single-GPU configuration
the 80%-of-HBM-roofline target is quoted on.  --scaling strong is configs[3]:
one 65536^2 grid split over the N GPUs (2-D Cartesian blocks by default, as
life_cart.c:117-124).  Inputs are generated on the device (counter-based
splitmix64, the same generator as oracle/life_oracle.c) and are resident in
HBM before timing.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--kernel bit|byte]
                  [--scaling weak|strong] [--size 65536]
                  [--workload random|p46gun_big] [--partition auto|cart|rows|cols]

Partition (life_dims_choose): "cart" (the default for both scalings) is
6-cartesian's MPI_Dims_create {2,1} / {2,2} / {4,2} split of life_cart.c:117-124
-- at N = 8 weak scaling that is the 262144 x 131072 global grid of
BASELINE configs[4] / SURVEY 8(d) C5, four halo peers per GPU; "rows" /
"auto" cut row strips {1, N} (the 1-D decomposition of 3-life/5-gather: two
peers, contiguous messages; measured 0-6 % cheaper per GPU with LOCAL
copies on one MI355X, not yet over xGMI), "cols" column strips.

N > 1 runs one process per GPU under torch.distributed.run: torch.distributed
(gloo) carries the bootstrap (RCCL unique id), the barriers and the
max-over-ranks timing; the halo data path is RCCL ncclSend/ncclRecv issued by
liblife_mi355x.so itself.  `--gpus N` without a launcher and with N GPUs
visible spawns those N rank processes itself (spawn_ranks) before any HIP
call; `--single-process` instead drives the N GPUs from one process
(ncclCommInitAll).  With fewer visible GPUs than --gpus the run is refused
unless --rehearse-shards is given: then one process runs the N shards with
device-local copies (how a 1-GPU box rehearses the partitioned schedule) and
the line says n_gpus = the devices actually used, config.shards = N.  Every
line carries config.devices (distinct PCI bus ids over all ranks) and
config.rccl_nranks (ncclCommCount).
`--shape WxH` replaces --size^2 (the per-GPU blocks of configs[3]).
Every N > 1 line ends with "phases" (mean ring / interior / halo / block
times per exchange, from HIP events on the three streams) and
"parity_vs_1gpu" (the N-shard grid against the same grid run as one shard).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "mpi-and-open-mp_amd"))

if int(os.environ.get("WORLD_SIZE", "1")) > 1 or "--rank-mode" in sys.argv:
    # torch bundles its own HIP runtime and links it by its unversioned name;
    # loading torch FIRST makes liblife_mi355x.so bind to that same runtime
    # (SONAME libamdhip64.so.7) instead of a second copy from /opt/rocm.
    import torch.distributed  # noqa: F401

import life_mi355x as lm  # noqa: E402  (the module; liblife_mi355x.so loads in main(), after spawn_ranks)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# VALU issue peak: 256 CUs x 4 SIMDs x 32 lanes/cycle (a wave64 instruction
# issues over 2 cycles, MI355X_MICROARCH.md "Wave scheduling") x 2.4 GHz.
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # defaults: one untimed launch, then generations 32..1024 of the random
    # soup (configs[2]/[4] run 1000 generations from the random start; a
    # multiple of both temporal depths, 16 and 32).  Launches get faster as the
    # soup thins out (profiles/r01/bench_warmup.jsonl); timing the whole run,
    # not only its cooled tail, keeps both in the rate.
    p.add_argument("--steps", type=int, default=992)
    p.add_argument("--warmup", type=int, default=32)
    p.add_argument("--kernel", default="bit", choices=["bit", "byte"])
    p.add_argument("--scaling", default="weak", choices=["weak", "strong"],
                   help="weak: a size^2 block per GPU (configs[4]); strong: one size^2 grid split over the GPUs "
                        "(configs[3])")
    p.add_argument("--size", type=int, default=65536,
                   help="block edge per GPU (weak) or global grid edge (strong)")
    p.add_argument("--shape", default=None, metavar="WxH",
                   help="a W x H block per GPU (weak) or global grid (strong) instead of --size^2: the per-GPU "
                        "blocks of configs[3] are 32768x65536 (N=2), 32768x32768 (N=4), 16384x32768 (N=8)")
    p.add_argument("--workload", default="random", choices=["random", "p46gun_big"])
    p.add_argument("--partition", default=None, choices=["auto", "cart", "rows", "cols"],
                   help="shard shape (life_dims_choose); default: cart (MPI_Dims_create, life_cart.c:117-118: "
                        "configs[3]'s and configs[4]'s 2-D split); auto = row strips when each is >= 1024 rows tall")
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="cpu_baseline sample budget (seconds of CPU work)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--parity-seconds", type=float, default=60.0,
                   help="N > 1: the 1-GPU reference re-runs the timed generations when that is estimated to take "
                        "less than this, else a fresh 3K+1-generation run of both")
    p.add_argument("--no-parity", action="store_true")
    p.add_argument("--rank-mode", action="store_true",
                   help="one-process-per-GPU set-up (gloo bootstrap, RCCL communicator) even at world 1")
    p.add_argument("--flow", type=int, default=None, choices=[0, 1, 2, 3],
                   help="LIFE_OPT_FLOW: single-shard bit tiles as one persistent dataflow launch per step call "
                        "(1 write-through, 2 fenced hand-off; 0 per-launch tiles; 3 automatic by rounds per pass; "
                        "default: the library's, 3)")
    p.add_argument("--no-overlap", action="store_true",
                   help="partitioned shards: every tile in one launch, then the halo exchange (LIFE_OPT_OVERLAP 0) "
                        "instead of ring / interior / halo on three streams")
    p.add_argument("--single-process", action="store_true",
                   help="--gpus N > 1 without a launcher: drive the N GPUs from this one process "
                        "(ncclCommInitAll) instead of spawning one process per GPU")
    p.add_argument("--rehearse-shards", action="store_true",
                   help="allow --gpus N above the visible GPU count: one process drives the N shards on the GPUs "
                        "there are (LOCAL device copies); the line then reports n_gpus = the devices actually used "
                        "and config.shards = N.  Without it such a run is refused")
    p.add_argument("--loopback-axes", default="xy", choices=["xy", "x", "y"],
                   help="--loopback: the axes exchanged through the transport (x: columns only, as N = 2's {2,1} "
                        "blocks; the other axis wraps in the stencil)")
    p.add_argument("--loopback", action="store_true",
                   help="N = 1: run the single grid as a periodic partition of itself (LIFE_OPT_LOOPBACK): the "
                        "halo exchange, ring / interior overlap and (with --rank-mode) RCCL send/recv of the "
                        "multi-GPU path, the shard its own neighbour")
    return p.parse_args()


def cpu_baseline(target_s: float):
    """The CPU oracle (a restatement of the reference's row-strip life_step,
    3-life/life_mpi.c:150-176, one OpenMP thread per strip) on a bounded
    sample of the same workload: a random 50% 4096^2 grid.  The reference's
    own mpirun rates were measured in the build container (the reference
    never travels to the GPU box) and are reported beside it as constants."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    n = 4096
    g = O.fill_random(n, n, 12345, 0.5)
    g = O.life_run(g, 1, threads)  # thread start-up and first touch, untimed
    # timed: doubling chunks of generations until the budget is spent (a
    # rate calibrated on a few generations was 3x off)
    gens, dt, chunk = 0, 0.0, 8
    while dt < target_s:
        t = time.perf_counter()
        g = O.life_run(g, chunk, threads)
        dt += time.perf_counter() - t
        gens += chunk
        per_gen = dt / gens
        chunk = max(1, min(2 * chunk, int((target_s - dt) / per_gen) + 1))
    return {"value": n * n * gens / dt / 1e9, "unit": "Gcell-updates/s", "cores": threads, "kind": "port",
            "sample": f"random 50% {n}x{n}, {gens} generations, oracle/life_oracle.c OpenMP row strips "
                      f"({threads} threads), {dt:.1f} s",
            "reference_mpirun_container": {
                "unit": "Gcell-updates/s", "cores": 8,
                "life_cart_np8_p46gun_big": 0.622, "life_cart_np8_random4096_steady": 0.357,
                "source": "BASELINE.md 'Re-measured in the survey container': reference 6-cartesian/life_cart.c, "
                          "gcc -O2, MPICH 3.3.2, mpiexec -n 8 on the build container's 8-core Xeon (not this host)"}}


def load_traffic(variant: str, size: str):
    """HBM bytes per stencil launch from the committed rocprofv3 PMC summary
    (scripts/traffic_summary.py); None where not measured for this variant."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as f:
            t = json.load(f)
        return t.get(f"{variant}_{size}")
    except (OSError, ValueError):
        return None


def make_life(a, nx, ny, dims, rank_mode, dist, rank, world, local_rank):
    if rank_mode:
        uid = [lm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        life = lm.Life.for_rank(nx, ny, rank, world, uid[0], local_rank, kernel=a.kernel, dims=dims)
    else:
        life = lm.Life(nx, ny, shards=a.gpus, kernel=a.kernel, dims=dims)
    if a.flow is not None:
        life.configure(lm.OPT_FLOW, a.flow)
    if a.no_overlap:
        life.configure(lm.OPT_OVERLAP, 0)
    return life


def topology(life, dist, world):
    """What the run actually used: the distinct physical
    GPUs (PCI bus ids) over every shard of every rank, and the rank count of
    the RCCL communicators (ncclCommCount; 0 = no communicator, LOCAL
    copies).  Collective in rank mode (gloo all_gather_object)."""
    infos = [life.shard_info(i) for i in range(life.world()["nlocal"])]
    if any(x is None for x in infos):
        return None
    buses = [x["pci_bus_id"] for x in infos]
    nranks = [x["rccl_nranks"] for x in infos]
    if dist is not None and world > 1:
        allb, alln = [None] * world, [None] * world
        dist.all_gather_object(allb, buses)
        dist.all_gather_object(alln, nranks)
        buses = [b for part in allb for b in part]
        nranks = [n for part in alln for n in part]
    lo, hi = min(nranks), max(nranks)
    return {"devices": len(set(buses)), "pci_bus_ids": sorted(set(buses)),
            "rccl_nranks": lo if lo == hi else [lo, hi]}


def init_grid(life, a, grid):
    if grid is not None:
        life.upload(grid)
    else:
        life.fill_random(a.seed, 0.5)


def parity_vs_1gpu(a, life, grid, nx, ny, gens_done, elapsed, n_gpus, rank, dist, barrier_sync):
    """The N-shard result against the same grid and generations run as ONE
    shard on GPU 0: the census checksum (sum of mix64(global index) over live
    cells, partition- and encoding-independent) and the live count.  The
    timed run's own end state is compared when re-running it on one GPU is
    estimated to take under --parity-seconds; otherwise both sides run a fresh
    3K+1 generations (several halo-exchange periods and a partial one)."""
    K = life.layout().generations_per_exchange
    same_run = elapsed * n_gpus * 1.3 < a.parity_seconds
    gens = gens_done
    if not same_run:
        gens = 3 * K + 1
        init_grid(life, a, grid)
        life.step(gens)
    got = (life.checksum(), life.live_count())  # collective in rank mode
    want = None
    if rank == 0:
        with lm.Life(nx, ny, shards=1, kernel=a.kernel) as ref:
            init_grid(ref, a, grid)
            ref.step(gens)
            want = (ref.checksum(), ref.live_count())
    barrier_sync()
    if rank != 0:
        return None
    return {"ok": got == want, "generations": gens, "same_run": same_run, "checksum": got[0], "live": got[1],
            "reference": {"checksum": want[0], "live": want[1], "shards": 1, "device": 0}}


def shape_of(a):
    """(W, H) of the workload: --shape WxH, else --size^2."""
    if a.shape:
        w, h = a.shape.lower().split("x")
        return int(w), int(h)
    return a.size, a.size


SHAPE_LABELS = {  # the single-GPU blocks the BASELINE configs put on one GPU
    (32768, 32768): "configs[2]; configs[3]'s N=4 block",
    (65536, 65536): "configs[4] weak scaling",
    (32768, 65536): "configs[3]'s N=2 block",
    (16384, 32768): "configs[3]'s N=8 block",
}


def visible_gpus() -> int:
    """GPUs this process may use, counted without initialising HIP (on this
    image torch.cuda.device_count() reads the topology only)."""
    try:
        import torch

        return int(torch.cuda.device_count())
    except Exception:  # noqa: BLE001 -- no torch / no ROCm: no GPUs to spawn for
        return 0


def spawn_ranks(n: int, argv, child=None) -> int:
    """One process per GPU (3-life/job_life.sh:7-8 runs one MPI rank per core):
    `bench.py --gpus N` without a launcher starts N children with RANK /
    WORLD_SIZE / LOCAL_RANK / MASTER_* set, exactly as torch.distributed.run
    would, and exits with the first failing rank's status.  The parent makes no HIP
    call before or after (it never loads liblife_mi355x.so); rank 0's JSON line
    is the one printed.  A single process driving N GPUs serialises ~28
    runtime calls per shard and exchange pass, more than a
    strong-scaling device pass."""
    import socket
    import subprocess

    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = child or [sys.executable, os.path.abspath(__file__), *argv]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(n), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen(cmd, env=env, stdout=None if r == 0 else sys.stderr))
    rcs = [None] * n
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
        bad = [rc for rc in rcs if rc not in (None, 0)]
        if bad:  # a dead rank leaves its peers waiting in a collective: stop them (our own children only)
            first = abs(bad[0])
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    p.terminate()
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    try:
                        rcs[i] = p.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        rcs[i] = p.wait()
            return first or 1
        time.sleep(0.05)
    return 0


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1 and "RANK" not in os.environ and a.gpus > 1 and not a.rank_mode:
        # no line may claim N GPUs it did not run on
        visible = visible_gpus()
        if visible >= a.gpus and not a.single_process:
            child = os.environ.get("LIFE_BENCH_CHILD_CMD")  # tests: a stand-in for the rank processes
            sys.exit(spawn_ranks(a.gpus, sys.argv[1:], json.loads(child) if child else None))
        if visible < a.gpus and not a.rehearse_shards:
            print(f"bench.py: --gpus {a.gpus} but {visible} GPU(s) visible; refusing to report an {a.gpus}-GPU line "
                  f"from fewer devices (pass --rehearse-shards to run {a.gpus} shards on the GPUs there are)",
                  file=sys.stderr, flush=True)
            sys.exit(2)
    lm._lib()
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    rank_mode = world > 1 or a.rank_mode
    if rank_mode:
        import torch.distributed as dist  # noqa: F811

        if world == 1 and "RANK" not in os.environ:
            # --rank-mode without a launcher: a world of one on this host
            import socket

            with socket.socket() as sk:
                sk.bind(("127.0.0.1", 0))
                port = sk.getsockname()[1]
            os.environ.update({"RANK": "0", "WORLD_SIZE": "1", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1",
                               "MASTER_PORT": str(port)})
        dist.init_process_group("gloo")
    n_gpus = world if world > 1 else a.gpus
    strong = a.scaling == "strong"
    partition = a.partition or "cart"
    W, H = shape_of(a)
    shape_txt = f"{W}^2" if W == H else f"{W}x{H}"
    grid = None
    if a.workload == "p46gun_big":
        _, _, grid = lm.load_cfg(os.path.join(ROOT, "tests", "golden", "cfg", "p46gun_big.cfg"))
        ny, nx = grid.shape
        dims = lm.dims_choose(nx, ny, n_gpus, partition)
        strong = True
        workload = "p46gun_big.cfg 500x500 (configs[1])"
    elif strong:
        nx, ny = W, H
        dims = lm.dims_choose(nx, ny, n_gpus, partition)
        workload = (f"random 50% {shape_txt} global, {dims[0]}x{dims[1]} blocks over {n_gpus} GPU(s) "
                    f"(configs[3] strong scaling)")
    else:
        # weak scaling: the shape is chosen for n_gpus blocks of W x H
        dims = lm.dims_choose(W, H * n_gpus, n_gpus, partition)
        nx, ny = W * dims[0], H * dims[1]
        label = SHAPE_LABELS.get((W, H), "weak scaling") if n_gpus == 1 else "configs[4] weak scaling"
        if n_gpus == 1 and (W, H) == (65536, 65536):
            label = "configs[4] at N=1 = the 65536^2 single-GPU roofline config"
        workload = f"random 50% {shape_txt} per GPU, global {nx}x{ny} ({label})"

    life = make_life(a, nx, ny, dims, rank_mode, dist, rank, world, local_rank)
    topo = topology(life, dist, world)
    init_grid(life, a, grid)
    if a.loopback:
        if n_gpus != 1:
            raise SystemExit("--loopback is a one-GPU mode")
        life.configure(lm.OPT_LOOPBACK, {"xy": 1, "x": 2, "y": 3}[a.loopback_axes])
    # The timed call of a single-stream step (one shard, no partitioned
    # axis: the N = 1 lines) carries one event pair around all its launches
    # (set_timing(2) keeps it so).  A multi-stream step (N > 1, --loopback)
    # is timed by its span only (set_timing(3)): per-launch events there put
    # ~10 us between back-to-back launches (profiles/r05/c, d).  Its kernel
    # statistics (the roofline object) and the overlapped schedule's phase
    # events (the "phases" object) are then recorded right after the timed
    # region, over K more generations (one exchange at least: with the deep
    # halo a short call may hold none), before anything else runs on the GPU:
    # recorded after the parity run and the copy-ceiling probe instead (round
    # 5), the same kernels ran 8-10 % faster than inside the timed call (the
    # GPU back at its idle clock; profiles/r06/a trace_loop96_oneshot: plain
    # passes 0.494-0.501 ms in the call, 0.454-0.457 ms in the statistics run),
    # so the phases understated the call's own blocks.
    # LIFE_BENCH_PHASES_TIMED=1 (or no warmup): all of it inside the timed call.
    phases_timed = os.environ.get("LIFE_BENCH_PHASES_TIMED", "0") == "1" or a.warmup <= 0
    multi = n_gpus > 1 or a.loopback
    stats_after = multi and not phases_timed
    life.set_timing(True)
    life.step(a.warmup)
    life.sync()

    def barrier_sync():
        # life.sync() = hipStreamSynchronize on every stream the library
        # launches on (the only GPU work in this process).  Rank mode: the
        # barrier is life_dev_barrier (an 8-byte RCCL all-reduce every rank
        # joins, then a stream sync: tens of us) rather than a gloo TCP
        # barrier, whose ~0.1-0.2 ms would sit inside a 20-generation timed
        # region; max-over-ranks goes through torch.distributed.
        if rank_mode:
            life.barrier()
        else:
            life.sync()

    life.set_timing(True if phases_timed else (3 if multi else 2))
    barrier_sync()
    t0 = time.perf_counter()
    life.step(a.steps)
    path = life.last_path()  # the kernel family of the timed call
    barrier_sync()
    elapsed = time.perf_counter() - t0

    def allmax(vals):
        if dist is None:
            return vals
        import torch

        t = torch.tensor(vals, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return [float(x) for x in t]

    call = life.call_stats()  # host enqueue / device span of the timed call
    elapsed, host_enq, pass_enq, span = allmax([elapsed, call["host_enqueue_ms"], call["pass_enqueue_max_ms"],
                                                call["device_span_ms"]])
    K = life.layout().generations_per_exchange
    if stats_after:
        life.set_timing(True)
        life.step(K)
        life.sync()
        ph = life.phase_stats()
    avg_ms, launches, bytes_per_launch = life.kernel_stats()
    updates_per_launch, valu_per_launch = life.kernel_work()
    if phases_timed:
        ph = life.phase_stats()
    live = life.live_count()
    lay = life.layout()
    temporal = lay.generations_per_exchange > 1

    # a measured stream-copy ceiling next to the spec peak
    # (rank 0's GPU, after the timed region; 2 x 2 GiB buffers)
    copy_gbps = lm.measure_copy(local_rank, 2 << 30, 5) if rank == 0 else 0.0

    parity = None
    if n_gpus > 1 and not a.no_parity:
        # the grid has advanced warmup + steps (+ K statistics generations)
        parity = parity_vs_1gpu(a, life, grid, nx, ny, a.warmup + a.steps + (K if stats_after else 0), elapsed,
                                n_gpus, rank, dist, barrier_sync)
    if multi:
        exposed = allmax([ph["block_ms"] - ph["interior_ms"], ph["block_ms"], ph["halo_ms"]])

    if rank == 0:
        cells = float(nx) * float(ny) * a.steps
        bpu = 0.25 if a.kernel == "bit" else 2.0  # algorithmic HBM bytes per cell-update
        value = cells / elapsed / 1e9
        hbm = bytes_per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
        gens_per_launch = updates_per_launch / (bytes_per_launch / bpu) if bytes_per_launch > 0 else 0.0
        variant = a.kernel + ("_temporal" if temporal else "_onegen")
        if path == "flow" and a.kernel == "bit":
            variant = "bit_flow"
        traffic = load_traffic(variant, shape_txt.replace("^2", "")) if (a.workload == "random" and not strong) else None
        # not measured by this run: the PMC pass of the same workload committed beside the code
        traffic_src = (f"profiles/traffic.json[{variant}_{shape_txt.replace('^2', '')}] (committed rocprofv3 "
                       "FETCH_SIZE x2 + WRITE_SIZE run of this workload, bytes per launch; not this run)"
                       if traffic is not None else None)
        hbm_obj = {"achieved": round(hbm, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                   "frac": round(hbm / HBM_PEAK_GBS, 4),
                   "bytes_per_launch": bytes_per_launch,
                   "copy_ceiling_GBps": round(copy_gbps, 1),
                   "frac_of_copy_ceiling": round(hbm / copy_gbps, 4) if copy_gbps > 0 else None,
                   # SURVEY 8(d)'s per-update figure (0.25 B bit / 2 B byte) x the
                   # cell-updates of a launch: above the HBM peak once a launch
                   # advances K > 1 generations per pass over HBM
                   "per_generation_equivalent_GBps": round(updates_per_launch * bpu / (avg_ms * 1e-3) / 1e9, 1)
                   if avg_ms > 0 else 0.0}
        tops = valu_per_launch / (avg_ms * 1e-3) / 1e12 if (valu_per_launch > 0 and avg_ms > 0) else 0.0
        if temporal and tops > 0:
            # the temporally blocked kernels are bound by VALU issue, not HBM.
            # achieved = ALGORITHMIC lane-ops per launch (the owned cells'
            # updates x the op count of the formulation: bit 22 per 64-cell
            # pair row and generation = 0.34375 per cell-update; byte 12 per
            # 32-cell word row and generation + 35 per word row and launch for
            # pack / unpack) over the mean launch time, against 256 CU x 4
            # SIMD x 32 lanes x 2.4 GHz.  "issued" adds what the tiling spends
            # on ghost rows and edge lanes (the kernel's op-count model as
            # tiled; SQ_INSTS_VALU is 2.7 % above it, profiles/r03/r5p).
            if a.kernel == "bit":
                algo = updates_per_launch * 22.0 / 64.0
            else:
                cells = updates_per_launch / gens_per_launch if gens_per_launch > 0 else 0.0
                algo = updates_per_launch * 12.0 / 32.0 + cells * 35.0 / 32.0
            useful = algo / (avg_ms * 1e-3) / 1e12
            roofline = {"bound": "valu", "achieved": round(useful, 2), "peak": round(VALU_PEAK_TOPS, 2),
                        "unit": "Tlane-op/s", "frac": round(useful / VALU_PEAK_TOPS, 4), "traffic": traffic,
                        "traffic_source": traffic_src,
                        "kernel_avg_ms": round(avg_ms, 5), "kernel_launches": launches,
                        "kernel_timing": ("HIP events on the launches of K generations after the timed call "
                                          "(a multi-stream call is timed by its span only)") if stats_after
                        else "HIP events on the timed call's stream",
                        "generations_per_launch": round(gens_per_launch, 3), "algorithmic_ops_per_launch": algo,
                        "issued": {"achieved": round(tops, 2), "frac": round(tops / VALU_PEAK_TOPS, 4),
                                   "ops_per_launch": valu_per_launch,
                                   "note": "op-count model of the launch as tiled (ghost rows, edge lanes, "
                                           "banded / half-height tiles included)"},
                        "model": "bit: per 64-cell pair row and generation 22 VALU (2 v_alignbit + 4 + 16 v_bitop3); "
                                 "byte: per 32-cell word row 12 per generation + 35 pack/unpack per launch; "
                                 "life_kernels.hip tile_body_bit / tile_body_byte",
                        "hbm": hbm_obj}
        else:
            roofline = dict(hbm_obj, bound="hbm", traffic=traffic, traffic_source=traffic_src, kernel_avg_ms=round(avg_ms, 5),
                            kernel_launches=launches, generations_per_launch=round(gens_per_launch, 3))
        out = {
            "metric": "Gcell-updates/sec at 1/2/4/8 MI355X + % of HBM roofline, bit-exact",
            "value": round(value, 3),
            "unit": "Gcell-updates/s",
            # the distinct GPUs the shards ran on (a --rehearse-shards run of
            # N shards on one GPU says 1 here and shards = N in config)
            "n_gpus": topo["devices"] if topo else n_gpus,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "u32 (1 bit/cell)" if a.kernel == "bit" else "u8 (1 byte/cell)",
            "data": "synthetic (device-side splitmix64 random, density 0.5)" if grid is None
                    else "p46gun_big.cfg pattern",
            "config": {"workload": workload, "nx": nx, "ny": ny, "dims": list(dims), "kernel": a.kernel,
                       "shards": n_gpus, "devices": topo["devices"] if topo else None,
                       "rccl_nranks": topo["rccl_nranks"] if topo else None,
                       "pci_bus_ids": topo["pci_bus_ids"] if topo else None,
                       "rehearsal": bool(topo and topo["devices"] < n_gpus),
                       "parallelism": f"cartesian {dims[0]}x{dims[1]}"
                                      + (" (one process per GPU, RCCL)" if rank_mode else
                                         f" ({life.world()['nlocal']} shards in one process, "
                                         f"{['auto', 'RCCL', 'LOCAL'][life.world()['transport']]} transport)"),
                       "partition": partition + (f" + loopback of axes {a.loopback_axes} (the shard its own neighbour)"
                                                 if a.loopback else ""), "kernel_path": path,
                       "generations_per_exchange": lay.generations_per_exchange, "live_cells_end": live},
            "roofline": roofline,
            # the timed call, self-diagnosing: CPU time
            # spent enqueueing it (whole call / longest pass), the device span
            # from its first work's start to its last work's end, and what the
            # bench clock saw outside that span (launch latency, host gaps, the
            # sync's wake-up); max over ranks
            "call": {"elapsed_ms": round(elapsed * 1e3, 4), "host_enqueue_ms": round(host_enq, 4),
                     "pass_enqueue_max_ms": round(pass_enq, 4), "passes": call["passes"],
                     "device_span_ms": round(span, 4),
                     "outside_span_ms": round(elapsed * 1e3 - span, 4) if span > 0 else None},
        }
        if n_gpus > 1 or a.loopback:
            out["phases"] = {"ring_ms": round(ph["ring_ms"], 4), "interior_ms": round(ph["interior_ms"], 4),
                             "halo_ms": round(ph["halo_ms"], 4), "block_ms": round(ph["block_ms"], 4),
                             "blocks": ph["blocks"], "exposed_ms": round(ph["block_ms"] - ph["interior_ms"], 4),
                             "max_over_ranks": {"exposed_ms": round(exposed[0], 4), "block_ms": round(exposed[1], 4),
                                                "halo_ms": round(exposed[2], 4)},
                             "note": "per overlapped block (one halo exchange): rank 0's shards; exposed = block - "
                                     "interior, the time the ring + halo add to the critical path; "
                                     + ("recorded in the timed call" if phases_timed else
                                        "recorded over K generations after the timed call (which carries no "
                                        "phase events)")}
        if parity is not None:
            out["parity_vs_1gpu"] = parity
        if n_gpus == 1 and not a.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(a.cpu_seconds)
        print(json.dumps(out), flush=True)
    life.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
