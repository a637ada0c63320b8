"""bench.py --gpus N without a launcher: one process per
GPU, spawned before the parent makes any HIP call, the way
torch.distributed.run would start them (3-life/job_life.sh:7-8 runs one MPI
rank per core).  CPU only: the rank processes are a stand-in script, the GPU
count is injected."""
import json
import os
import subprocess
import sys

import torch  # noqa: F401  (before any test loads liblife_mi355x: the gloo test spawns through torch)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PARENT = """
import sys
sys.path.insert(0, {root!r})
import bench
bench.visible_gpus = lambda: {ngpu}
sys.argv = ["bench.py", "--gpus", "{n}", "--steps", "3"] + {extra!r}
rc = 0
try:
    bench.main()
except SystemExit as e:
    rc = e.code
maps = open("/proc/self/maps").read()
assert "liblife_mi355x" not in maps, "the parent loaded the library"
print("PARENT_RC", rc, flush=True)
"""

CHILD = """
import json, os, sys, time
r, n = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
assert os.environ["LOCAL_RANK"] == str(r) and os.environ["MASTER_ADDR"] == "127.0.0.1"
assert int(os.environ["MASTER_PORT"]) > 0
assert sys.argv[1:] == ["--gpus", str(n), "--steps", "3"], sys.argv
if os.environ.get("FAIL_RANK") == str(r):
    sys.exit(3)
if os.environ.get("FAIL_RANK"):
    time.sleep(60)  # a rank waiting for a dead peer: the parent must stop it
if r == 0:
    print(json.dumps({"metric": "stand-in", "rank": r, "world": n}), flush=True)
else:
    print("rank", r, "quiet", flush=True)
"""


def _run(tmp_path, n, ngpu, fail_rank=None, extra=()):
    child = tmp_path / "child.py"
    child.write_text(CHILD)
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["LIFE_BENCH_CHILD_CMD"] = json.dumps([sys.executable, str(child), "--gpus", str(n), "--steps", "3"])
    if fail_rank is not None:
        env["FAIL_RANK"] = str(fail_rank)
    return subprocess.run([sys.executable, "-c", PARENT.format(root=ROOT, n=n, ngpu=ngpu, extra=list(extra))], env=env,
                          capture_output=True, text=True, timeout=120)


def test_spawns_one_process_per_gpu(tmp_path):
    out = _run(tmp_path, 3, 8)
    assert "PARENT_RC 0" in out.stdout, out.stderr
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert [json.loads(ln) for ln in lines] == [{"metric": "stand-in", "rank": 0, "world": 3}]
    assert "rank 2 quiet" in out.stderr  # the other ranks' stdout goes to stderr


def test_dead_rank_stops_the_others(tmp_path):
    out = _run(tmp_path, 4, 4, fail_rank=1)
    assert "PARENT_RC 3" in out.stdout, out.stdout + out.stderr


def test_fewer_gpus_than_ranks_is_refused(tmp_path):
    """with fewer visible GPUs than --gpus (and no
    --rehearse-shards) the run stops before the library loads, with a
    non-zero status, instead of printing an N-GPU line from fewer devices."""
    out = _run(tmp_path, 8, 1)
    assert "stand-in" not in out.stdout
    assert "PARENT_RC 2" in out.stdout, out.stdout + out.stderr
    assert "--rehearse-shards" in out.stderr


def test_single_process_with_fewer_gpus_is_refused(tmp_path):
    out = _run(tmp_path, 4, 2, extra=["--single-process"])
    assert "PARENT_RC 2" in out.stdout, out.stdout + out.stderr


def test_rehearse_shards_stays_in_process(tmp_path):
    """--rehearse-shards: nothing is spawned, the parent goes on to drive N
    LOCAL shards, which here (no GPU) fails in the library after it was
    loaded (so the script's no-library assertion is never reached)."""
    out = _run(tmp_path, 8, 1, extra=["--rehearse-shards"])
    assert "stand-in" not in out.stdout
    assert "PARENT_RC" not in out.stdout
    assert "refusing" not in out.stderr


def test_topology_counts_distinct_devices():
    """n_gpus / config.devices come from the shards' PCI bus ids, not from
    --gpus: 8 LOCAL shards on one GPU are one device."""
    sys.path.insert(0, ROOT)
    import bench

    class FakeLife:
        def __init__(self, buses, nranks):
            self.buses, self.nranks = buses, nranks

        def world(self):
            return {"nlocal": len(self.buses)}

        def shard_info(self, i):
            return {"device": 0, "pci_bus_id": self.buses[i], "rccl_nranks": self.nranks[i]}

    t = bench.topology(FakeLife(["0000:05:00.0"] * 8, [0] * 8), None, 1)
    assert t == {"devices": 1, "pci_bus_ids": ["0000:05:00.0"], "rccl_nranks": 0}
    t = bench.topology(FakeLife([f"0000:{i:02x}:00.0" for i in range(4)], [4] * 4), None, 1)
    assert t["devices"] == 4 and t["rccl_nranks"] == 4
    t = bench.topology(FakeLife(["a", "b"], [2, 1]), None, 1)
    assert t["rccl_nranks"] == [1, 2]


def _topo_worker(rank, world, port, q):
    import torch.distributed as dist

    sys.path.insert(0, ROOT)
    import bench

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)

    class OneShard:  # one process per GPU: one shard each, its own device
        def world(self):
            return {"nlocal": 1}

        def shard_info(self, i):
            return {"device": 0, "pci_bus_id": f"0000:{0x10 + rank:02x}:00.0", "rccl_nranks": world}

    q.put((rank, bench.topology(OneShard(), dist, world)))
    dist.destroy_process_group()


def test_topology_over_gloo_world2():
    """Rank mode: the devices of every rank are gathered (gloo), so a
    2-rank job on two GPUs reports devices 2 and rccl_nranks 2 on rank 0."""
    import socket

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_topo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert got[0] == got[1] == {"devices": 2, "pci_bus_ids": ["0000:10:00.0", "0000:11:00.0"], "rccl_nranks": 2}
