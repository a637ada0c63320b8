"""Multi-rank halo exchange on CPU: world_size 2/4/8 processes over gloo
execute the product's halo plan (life_halo_plan, the same ops the RCCL
transport issues, matched in issue order per peer like ncclSend/ncclRecv) on
apron-padded blocks, step each block with the oracle, and must reproduce
the single-grid oracle bit for bit.  This is the N>1 path of
life_dev_step minus the device: partition, neighbour table, op order,
corner propagation through width+2 rows."""
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


def _worker(rank, world, port, nx, ny, dims, gens, seed, q):
    try:
        sys.path.insert(0, os.path.join(ROOT, "mpi-and-open-mp_amd"))
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import life_mi355x as lm
        import oracle as O

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        full = O.fill_random(nx, ny, seed, 0.45)
        L = lm.layout_query(nx, ny, dims, rank)
        w, h = L.w, L.h
        P = np.zeros((h + 2, w + 2), np.uint8)  # P[y+1, x+1] = cell(x, y)
        P[1:h + 1, 1:w + 1] = full[L.y0:L.y0 + h, L.x0:L.x0 + w]
        plan = lm.halo_plan(nx, ny, dims, rank)

        def region(o):
            _, _, _, what, index, first, count = o
            if what == lm.HALO_COLUMN:
                return (slice(first, first + count), index + 1)
            return (index, slice(first + 1, first + 1 + count))

        def exchange():
            for phase in (0, 1):
                ops = [o for o in plan if o[0] == phase]
                if ops[0][1] == lm.HALO_FILL:  # axis inside the shard: periodic wrap
                    if phase == 0:
                        P[1:h + 1, 0] = P[1:h + 1, w]
                        P[1:h + 1, w + 1] = P[1:h + 1, 1]
                    else:
                        P[0, :] = P[h, :]
                        P[h + 1, :] = P[1, :]
                    continue
                sent, recvd, reqs, bufs = {}, {}, [], []
                for o in ops:  # k-th message between a pair = tag k (RCCL: issue order)
                    peer = o[2]
                    if o[1] == lm.HALO_SEND:
                        k = sent.get(peer, 0)
                        sent[peer] = k + 1
                        t = torch.from_numpy(np.ascontiguousarray(P[region(o)]))
                        reqs.append(dist.isend(t, peer, tag=k))
                    else:
                        k = recvd.get(peer, 0)
                        recvd[peer] = k + 1
                        t = torch.empty(o[6], dtype=torch.uint8)
                        reqs.append(dist.irecv(t, peer, tag=k))
                        bufs.append((o, t))
                for r in reqs:
                    r.wait()
                for o, t in bufs:
                    P[region(o)] = t.numpy()

        exchange()
        for _ in range(gens):
            P[:] = O.step_padded(P, w, h)
            exchange()
        q.put((rank, L.x0, L.y0, P[1:h + 1, 1:w + 1].copy()))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # surface worker failures to the parent
        q.put((rank, "error", repr(e), None))
        raise


@pytest.mark.parametrize("world,nx,ny,gens", [(2, 23, 17, 6), (4, 20, 9, 7), (8, 33, 10, 5), (3, 7, 11, 4),
                                              (8, 4, 2, 3), (6, 31, 25, 5)])
def test_plan_over_gloo(oracle, lm, world, nx, ny, gens):
    dims = lm.dims_create(world)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, nx, ny, dims, gens, 42 + world, q))
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
