"""bench.py --gpus N without a launcher: one process per
GPU, spawned before the parent makes any HIP call, the way
torch.distributed.run would start them (3-life/job_life.sh:7-8 runs one MPI
rank per core).  CPU only: the rank processes are a stand-in script, the GPU
count is injected."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

PARENT = """
import sys
sys.path.insert(0, {root!r})
import bench
bench.visible_gpus = lambda: {ngpu}
sys.argv = ["bench.py", "--gpus", "{n}", "--steps", "3"]
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


def _run(tmp_path, n, ngpu, fail_rank=None):
    child = tmp_path / "child.py"
    child.write_text(CHILD)
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["LIFE_BENCH_CHILD_CMD"] = json.dumps([sys.executable, str(child), "--gpus", str(n), "--steps", "3"])
    if fail_rank is not None:
        env["FAIL_RANK"] = str(fail_rank)
    return subprocess.run([sys.executable, "-c", PARENT.format(root=ROOT, n=n, ngpu=ngpu)], env=env,
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


def test_fewer_gpus_than_ranks_stays_in_process(tmp_path):
    """With fewer visible GPUs than --gpus (the one-GPU box rehearsing N
    shards) nothing is spawned: the parent goes on to drive LOCAL shards,
    which here (no GPU) fails in the library, after it was loaded."""
    out = _run(tmp_path, 8, 1)
    assert "stand-in" not in out.stdout
    assert "PARENT_RC" not in out.stdout  # the in-process path got past the spawn check and failed on no GPU
