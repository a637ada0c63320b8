#!/usr/bin/env python3
"""Benchmark of the MI355X Game-of-Life hot path (one JSON line on rank 0).

A "step" is one generation (halo exchange + B3/S23 update) over the whole
grid.  Default workload (BASELINE.json configs[4], weak scaling): a random
50%-density 65536 x 65536 block per GPU, global grid
(65536*dims0) x (65536*dims1) (dims: --partition below); N = 1 is the
65536^2 single-GPU configuration the 80%-of-HBM-roofline target is quoted on.
Inputs are generated on the device (counter-based splitmix64, the same
generator as oracle/life_oracle.c) and are resident in HBM before timing.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--kernel bit|byte]
                  [--size 65536] [--workload weak|p46gun_big]
                  [--partition auto|cart|rows|cols]

Partition (life_dims_choose): "auto" (default) cuts the global grid into
row strips, dims {1, N} (the 1-D decomposition of 3-life/5-gather), because
measured per-GPU cost is 0-6 % lower than for 2-D blocks and every halo
message is contiguous; "cart" is 6-cartesian's MPI_Dims_create {2,1} /
{2,2} / {4,2}.  Either way each GPU owns one size x size block.

N > 1 runs one process per GPU under torch.distributed.run: torch.distributed
(gloo) carries the bootstrap (RCCL unique id), the barriers and the
max-over-ranks timing; the halo data path is RCCL ncclSend/ncclRecv issued by
liblife_mi355x.so itself.
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

import life_mi355x as lm  # noqa: E402

lm._lib()

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip-level parameters)
# VALU issue peak: 256 CUs x 4 SIMDs x 32 lanes/cycle (a wave64 instruction
# issues over 2 cycles, MI355X_MICROARCH.md "Wave scheduling") x 2.4 GHz.
VALU_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    # defaults: whole multiples of the temporal kernel's 32 generations per
    # launch; one untimed launch, then generations 32..1024 of the random soup
    # (configs[2]/[4] run 1000 generations from the random start).  Launches
    # get faster as the soup thins out (65536^2 bit: 1.61 ms per launch at
    # the start, 1.36 ms after ~10 launches, profiles/r01/bench_warmup.jsonl);
    # timing the whole run, not only its cooled tail, keeps both in the rate.
    p.add_argument("--steps", type=int, default=992)
    p.add_argument("--warmup", type=int, default=32)
    p.add_argument("--kernel", default="bit", choices=["bit", "byte"])
    p.add_argument("--size", type=int, default=65536, help="per-GPU block edge (weak scaling)")
    p.add_argument("--workload", default="weak", choices=["weak", "p46gun_big"])
    p.add_argument("--partition", default="auto", choices=["auto", "cart", "rows", "cols"],
                   help="shard shape (life_dims_choose): auto = row strips when each is >= 1024 rows tall")
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--cpu-seconds", type=float, default=10.0, help="cpu_baseline sample budget")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--temporal", default="tiles", choices=["sweep", "tiles"],
                   help="temporally blocked kernel: the tiled tstep_kernel (default) or sweep_kernel")
    p.add_argument("--rank-mode", action="store_true",
                   help="one-process-per-GPU set-up (gloo bootstrap, RCCL communicator) even at world 1")
    return p.parse_args()


def cpu_baseline(target_s: float):
    """The CPU oracle (a restatement of the reference's row-strip life_step,
    3-life/life_mpi.c:150-176, one OpenMP thread per strip) on a bounded
    sample of the same workload: a random 50% 4096^2 grid."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    n = 4096
    g = O.fill_random(n, n, 12345, 0.5)
    t = time.perf_counter()
    g = O.life_run(g, 1, threads)
    one = max(time.perf_counter() - t, 1e-6)
    gens = max(1, int(target_s / one))
    t = time.perf_counter()
    O.life_run(g, gens, threads)
    dt = time.perf_counter() - t
    res = {"value": n * n * gens / dt / 1e9, "unit": "Gcell-updates/s", "cores": threads, "kind": "port",
           "sample": f"random 50% {n}x{n}, {gens} generations, oracle/life_oracle.c OpenMP row strips, "
                     f"{dt:.1f} s"}
    ref = O.ref_lib()
    if ref is not None:  # the reference's own life_step (3-life/life2d.c), when built
        m = 2048
        g2 = O.fill_random(m, m, 12345, 0.5)
        t = time.perf_counter()
        O.ref_life_run(g2, 2)
        dt2 = time.perf_counter() - t
        res["reference_1core"] = {"value": m * m * 2 / dt2 / 1e9, "unit": "Gcell-updates/s",
                                  "sample": f"random 50% {m}x{m}, 2 generations, reference life_step "
                                            "(3-life/life2d.c:104-130, gcc -O2), 1 core"}
    return res


def load_traffic(variant: str, size: int):
    """HBM bytes per stencil launch from the committed rocprofv3 PMC summary
    (scripts/traffic_summary.py); None where the access width is uncalibrated."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        with open(path) as f:
            t = json.load(f)
        return t.get(f"{variant}_{size}")
    except (OSError, ValueError):
        return None


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    rank_mode = world > 1 or a.rank_mode
    if rank_mode:
        import torch.distributed as dist  # noqa: F811

        dist.init_process_group("gloo")
    n_gpus = world if world > 1 else a.gpus
    if a.workload == "p46gun_big":
        steps_cfg, _, grid = lm.load_cfg(os.path.join(ROOT, "tests", "golden", "cfg", "p46gun_big.cfg"))
        ny, nx = grid.shape
        dims = lm.dims_choose(nx, ny, n_gpus, a.partition)
        workload = "p46gun_big.cfg 500x500 (configs[1])"
    else:
        # weak scaling: the shape is chosen for n_gpus blocks of size^2 stacked as strips
        dims = lm.dims_choose(a.size, a.size * n_gpus, n_gpus, a.partition)
        nx, ny = a.size * dims[0], a.size * dims[1]
        grid = None
        workload = f"random 50% {a.size}^2 per GPU, global {nx}x{ny} (configs[4] weak scaling)"

    if rank_mode:
        uid = [lm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        life = lm.Life.for_rank(nx, ny, rank, world, uid[0], local_rank, kernel=a.kernel, dims=dims)
    else:
        life = lm.Life(nx, ny, shards=a.gpus, kernel=a.kernel, dims=dims)
    if a.temporal == "sweep":
        life.configure(lm.OPT_SWEEP, 1)

    if grid is not None:
        life.upload(grid)
    else:
        life.fill_random(a.seed, 0.5)
    life.step(a.warmup)
    life.sync()

    def barrier_sync():
        # life.sync() = hipStreamSynchronize on every stream the library
        # launches on (the only GPU work in this process); the barrier and
        # max-over-ranks go through torch.distributed when N > 1.
        life.sync()
        if dist is not None:
            dist.barrier()

    life.set_timing(True)
    barrier_sync()
    t0 = time.perf_counter()
    life.step(a.steps)
    barrier_sync()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        import torch

        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    avg_ms, launches, bytes_per_launch = life.kernel_stats()
    updates_per_launch, valu_per_launch = life.kernel_work()
    live = life.live_count()

    # a measured stream-copy ceiling next to the spec peak
    # (rank 0's GPU, after the timed region; 2 x 2 GiB buffers)
    copy_gbps = lm.measure_copy(local_rank, 2 << 30, 5) if rank == 0 else 0.0

    if rank == 0:
        cells = float(nx) * float(ny) * a.steps
        bpu = 0.25 if a.kernel == "bit" else 2.0  # algorithmic HBM bytes per cell-update
        value = cells / elapsed / 1e9
        achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
        gens_per_launch = updates_per_launch / (bytes_per_launch / (0.25 if a.kernel == "bit" else 2.0)) \
            if bytes_per_launch > 0 else 0.0
        temporal = life.layout().generations_per_exchange > 1
        variant = a.kernel + ("_temporal" if temporal else "_onegen")
        traffic = load_traffic(variant, a.size) if a.workload == "weak" else None
        out = {
            "metric": "Gcell-updates/sec at 1/2/4/8 MI355X + % of HBM roofline, bit-exact",
            "value": round(value, 3),
            "unit": "Gcell-updates/s",
            "n_gpus": n_gpus,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32 (1 bit/cell)" if a.kernel == "bit" else "u8 (1 byte/cell)",
            "data": "synthetic (device-side splitmix64 random, density 0.5)" if grid is None
                    else "p46gun_big.cfg pattern",
            "config": {"workload": workload, "nx": nx, "ny": ny, "dims": list(dims), "kernel": a.kernel,
                       "parallelism": f"cartesian {dims[0]}x{dims[1]}", "partition": a.partition,
                       "live_cells_end": live},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel_avg_ms": round(avg_ms, 5), "kernel_launches": launches,
                         "bytes_per_launch": bytes_per_launch,
                         "generations_per_launch": round(gens_per_launch, 3),
                         # SURVEY 8(d)'s per-update figure (0.25 B bit / 2 B byte) x the
                         # cell-updates of a launch: above the HBM peak once a launch
                         # advances K > 1 generations per pass over HBM
                         "per_generation_equivalent_GBps": round(
                             updates_per_launch * (0.25 if a.kernel == "bit" else 2.0) / (avg_ms * 1e-3) / 1e9, 1)
                         if avg_ms > 0 else 0.0,
                         # the north-star question "% of HBM roofline" in cell-update terms: the
                         # rate a one-generation-per-HBM-pass kernel would reach at the HBM peak on
                         # n_gpus GPUs (8 TB/s / 0.25 B or 2 B per update), and value against it
                         "copy_ceiling_GBps": round(copy_gbps, 1),
                         "frac_of_copy_ceiling": round(achieved / copy_gbps, 4) if copy_gbps > 0 else None,
                         "hbm_bound_cell_rate": round(n_gpus * HBM_PEAK_GBS / bpu, 1),
                         "cell_rate_vs_hbm_bound": round(value / (n_gpus * HBM_PEAK_GBS / bpu), 4)},
        }
        if valu_per_launch > 0 and avg_ms > 0:
            # the temporally blocked kernel is VALU-issue bound, not HBM bound
            tops = valu_per_launch / (avg_ms * 1e-3) / 1e12
            out["valu"] = {"bound": "valu", "achieved": round(tops, 2), "peak": round(VALU_PEAK_TOPS, 2),
                           "unit": "Tlane-op/s", "frac": round(tops / VALU_PEAK_TOPS, 4),
                           "ops_per_launch": valu_per_launch, "model": "13 VALU ops per register row "
                           "and generation + byte pack/unpack (life_kernels.hip tstep_valu_per_tile_lane), "
                           "within 2% of SQ_INSTS_VALU (profiles/r01/pmc_SQ_*_temporal.csv)"}
        if n_gpus == 1 and not a.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(a.cpu_seconds)
        print(json.dumps(out), flush=True)
    life.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
