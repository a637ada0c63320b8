"""Multi-rank halo exchange on CPU: world_size 2/4/8 processes over gloo
execute the product's halo plan (life_halo_plan, the same ops the RCCL
transport issues, matched in issue order per peer like ncclSend/ncclRecv) on
apron-padded blocks, step each block with the oracle, and must reproduce
the single-grid oracle bit for bit.  This is the N>1 path of
life_dev_step minus the device: partition, neighbour table, op order,
corners through width+2 rows (one-cell aprons) or as explicit K x xapron
blocks of the one-phase plan (temporal aprons, both axes partitioned), whose
receives land after the rows' stale apron bytes."""
import os
import socket
import sys

import numpy as np
import pytest

import torch  # noqa: F401  (load torch before liblife_mi355x: one HIP runtime per process)
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, nx, ny, dims, gens, seed, kernel, q):
    try:
        sys.path.insert(0, os.path.join(ROOT, "mpi-and-open-mp_amd"))
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import life_mi355x as lm
        import oracle as O

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        full = O.fill_random(nx, ny, seed, 0.45)
        L = lm.layout_query(nx, ny, dims, rank, kernel)
        w, h, xa, ya, gpe = L.w, L.h, L.xapron, L.yapron, L.generations_per_exchange
        # cell (x, y) at P[y + ya, x + xa]: the device layout's cell frame
        P = np.zeros((h + 2 * ya, w + 2 * xa), np.uint8)
        P[ya:ya + h, xa:xa + w] = full[L.y0:L.y0 + h, L.x0:L.x0 + w]
        plan = lm.halo_plan(nx, ny, dims, rank, kernel)

        def region(o):
            _, _, _, what, index, first, count, width = o
            if what in (lm.HALO_COLUMN, lm.HALO_CORNER):
                return (slice(first, first + count), slice(index + xa, index + xa + width))
            return (slice(index, index + width), slice(first + xa, first + xa + count))

        def exchange():
            for phase in (0, 1):
                ops = [o for o in plan if o[0] == phase]
                if not ops:  # the fused one-phase plan (both axes, temporal aprons)
                    continue
                if ops[0][1] == lm.HALO_FILL:  # axis inside the shard: periodic wrap
                    if phase == 0:
                        P[ya:ya + h, :] = P[ya:ya + h, xa + np.arange(-xa, w + xa) % w]
                    else:
                        P[:, :] = P[ya + np.arange(-ya, h + ya) % h, :]
                    continue
                sent, recvd, reqs, bufs = {}, {}, [], []
                for o in ops:  # k-th message between a pair = tag k (RCCL: issue order)
                    peer = o[2]
                    if o[1] == lm.HALO_SEND:
                        k = sent.get(peer, 0)
                        sent[peer] = k + 1
                        t = torch.from_numpy(np.ascontiguousarray(P[region(o)]).reshape(-1))
                        reqs.append(dist.isend(t, peer, tag=k))
                    else:
                        k = recvd.get(peer, 0)
                        recvd[peer] = k + 1
                        t = torch.empty(o[6] * o[7], dtype=torch.uint8)
                        reqs.append(dist.irecv(t, peer, tag=k))
                        bufs.append((o, t))
                for r in reqs:
                    r.wait()
                for o, t in bufs:
                    P[region(o)] = t.numpy().reshape(P[region(o)].shape)

        exchange()
        done = 0
        while done < gens:
            m = min(gpe, gens - done)
            for _ in range(m):  # the padded block as its own grid: wrong values
                P[:] = O.np_life_step(P)  # creep in from its border one cell per generation
            done += m
            exchange()
        q.put((rank, L.x0, L.y0, P[ya:ya + h, xa:xa + w].copy()))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # surface worker failures to the parent
        q.put((rank, "error", repr(e), None))
        raise


@pytest.mark.parametrize("kernel,world,nx,ny,gens", [
    ("byte", 2, 23, 17, 6), ("byte", 4, 20, 9, 7), ("byte", 8, 33, 10, 5), ("byte", 3, 7, 11, 4),
    ("byte", 8, 4, 2, 3), ("byte", 6, 31, 25, 5), ("byte", 4, 64, 40, 35), ("byte", 2, 64, 16, 20), ("byte", 4, 64, 80, 70),
    ("bit", 2, 64, 20, 19), ("bit", 4, 64, 16, 17), ("bit", 8, 128, 16, 12), ("bit", 3, 96, 9, 9),
    ("bit", 4, 70, 20, 5), ("bit", 4, 64, 40, 35), ("bit", 8, 128, 36, 20), ("bit", 2, 96, 34, 33),
    ("bit", 4, 64, 80, 70), ("bit", 8, 128, 64, 40),
])
def test_plan_over_gloo(oracle, lm, kernel, world, nx, ny, gens):
    """Either encoding: 32-cell x /
    K-row y aprons, up to K = 32 generations per exchange (temporal layouts),
    or the one-cell fallback when a block width is not a multiple of 32 or a
    partitioned block is shorter than K rows."""
    dims = lm.dims_create(world)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nx, ny, dims, gens, 42 + world, kernel, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = np.full((ny, nx), 255, np.uint8)
    for _ in range(world):
        rank, x0, y0, block = q.get(timeout=120)
        assert x0 != "error", f"rank {rank}: {y0}"
        got[y0:y0 + block.shape[0], x0:x0 + block.shape[1]] = block
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = oracle.life_run(oracle.fill_random(nx, ny, 42 + world, 0.45), gens)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("kernel,world,nx,ny,gens", [
    ("bit", 2, 96, 64, 40), ("bit", 4, 64, 4 * 33, 33), ("bit", 8, 64, 8 * 40, 37),
    ("byte", 2, 64, 70, 35), ("byte", 4, 40, 16, 5), ("byte", 8, 64, 8 * 32, 34),
])
def test_row_strips_over_gloo(oracle, lm, kernel, world, nx, ny, gens):
    """The 1-D row-strip partition (life_dims_choose "rows", dims {1, world}):
    every message is a run of whole padded rows, up and down the ring, as in
    5-gather/life_mpi.c:181-191 but K rows deep for the temporal layouts."""
    dims = lm.dims_choose(nx, ny, world, "rows")
    assert dims == (1, world)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nx, ny, dims, gens, 7 + world, kernel, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = np.full((ny, nx), 255, np.uint8)
    for _ in range(world):
        rank, x0, y0, block = q.get(timeout=120)
        assert x0 != "error", f"rank {rank}: {y0}"
        got[y0:y0 + block.shape[0], x0:x0 + block.shape[1]] = block
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = oracle.life_run(oracle.fill_random(nx, ny, 7 + world, 0.45), gens)
    np.testing.assert_array_equal(got, want)
