"""The driver's launcher support (driver/bootstrap.c), on the CPU: rank
variables of torchrun / MPICH / Open MPI are recognised, and the 128-byte
RCCL unique id travels from rank 0 to every other rank over TCP.  A small C
harness links bootstrap.c alone (no HIP)."""
import os
import socket
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRV = os.path.join(ROOT, "mpi-and-open-mp_amd", "driver")

HARNESS = r"""
#include <stdio.h>
#include <string.h>
#include "bootstrap.h"
int main(void) {
    int rank, world, local;
    const int found = life_launcher_ranks(&rank, &world, &local);
    if (found != 1) { printf("found %d\n", found); return 0; }
    uint8_t id[LIFE_UID_BYTES];
    memset(id, 0, sizeof id);
    if (rank == 0) for (int k = 0; k < LIFE_UID_BYTES; k++) id[k] = (uint8_t)(k * 7 + 3);
    const int rc = life_bootstrap_id(rank, world, id, 20.0);
    printf("rank %d world %d local %d rc %d id", rank, world, local, rc);
    for (int k = 0; k < LIFE_UID_BYTES; k += 16) printf(" %02x", id[k]);
    printf("\n");
    return rc ? 1 : 0;
}
"""


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    d = tmp_path_factory.mktemp("boot")
    (d / "h.c").write_text(HARNESS)
    exe = d / "h"
    subprocess.run(["gcc", "-O1", "-Wall", f"-I{DRV}", str(d / "h.c"), os.path.join(DRV, "bootstrap.c"), "-o",
                    str(exe)], check=True)
    return str(exe)


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def clean_env(**kv):
    env = {k: v for k, v in os.environ.items()
           if not k.startswith(("RANK", "WORLD_SIZE", "LOCAL_RANK", "PMI_", "OMPI_", "MPI_LOCALRANKID",
                                "MASTER_", "LIFE_BOOTSTRAP"))}
    env.update({k: str(v) for k, v in kv.items()})
    return env


@pytest.mark.parametrize("style", ["torchrun", "mpich", "openmpi"])
def test_id_reaches_every_rank(harness, style):
    world, port = 4, free_port()
    names = {"torchrun": ("RANK", "WORLD_SIZE", "LOCAL_RANK"), "mpich": ("PMI_RANK", "PMI_SIZE", "MPI_LOCALRANKID"),
             "openmpi": ("OMPI_COMM_WORLD_RANK", "OMPI_COMM_WORLD_SIZE", "OMPI_COMM_WORLD_LOCAL_RANK")}[style]
    procs = []
    for r in (3, 1, 2, 0):  # rank 0 last: the others retry until it listens
        env = clean_env(**{names[0]: r, names[1]: world, names[2]: r}, LIFE_BOOTSTRAP_PORT=port)
        procs.append(subprocess.Popen([harness], env=env, stdout=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=60)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    ids = {o.split(" id ")[1].strip() for o in outs}
    assert len(ids) == 1 and ids.pop().startswith("03 73")  # id[0] = 3, id[16] = 115 from rank 0
    assert sorted(int(o.split()[1]) for o in outs) == [0, 1, 2, 3]


def test_no_launcher_and_bad_values(harness):
    r = subprocess.run([harness], env=clean_env(), capture_output=True, text=True, timeout=30)
    assert r.stdout.strip() == "found 0"
    r = subprocess.run([harness], env=clean_env(RANK=4, WORLD_SIZE=4), capture_output=True, text=True, timeout=30)
    assert r.stdout.strip() == "found -1"


def test_master_port_plus_one(harness):
    """torchrun's MASTER_ADDR / MASTER_PORT: the id goes over MASTER_PORT + 1."""
    port = free_port()
    procs = [subprocess.Popen([harness], env=clean_env(RANK=r, WORLD_SIZE=2, MASTER_ADDR="127.0.0.1",
                                                         MASTER_PORT=port - 1), stdout=subprocess.PIPE, text=True)
             for r in (1, 0)]
    outs = [p.communicate(timeout=60)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    assert outs[0].split(" id ")[1] == outs[1].split(" id ")[1]


def test_master_addr_hostname(harness):
    """torchrun --standalone exports a host NAME as MASTER_ADDR; "localhost"
    resolves through getaddrinfo (inet_pton accepted only dotted
    quads)."""
    port = free_port()
    procs = [subprocess.Popen([harness], env=clean_env(RANK=r, WORLD_SIZE=2, MASTER_ADDR="localhost",
                                                         MASTER_PORT=port - 1), stdout=subprocess.PIPE, text=True)
             for r in (1, 0)]
    outs = [p.communicate(timeout=60)[0] for p in procs]
    assert all(p.returncode == 0 for p in procs), outs
    assert outs[0].split(" id ")[1] == outs[1].split(" id ")[1]


def test_rank0_times_out_when_a_rank_never_connects(harness):
    """Rank 0 of a 2-rank job whose rank 1 never starts: the accept wait is
    bounded by the timeout (20 s in the harness) and fails, not a hang."""
    import time

    t = time.monotonic()
    r = subprocess.run([harness], env=clean_env(RANK=0, WORLD_SIZE=2, LIFE_BOOTSTRAP_PORT=free_port()),
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and " rc -1 " in r.stdout, r.stdout
    assert 15 < time.monotonic() - t < 45


def test_stranger_neither_gets_the_id_nor_a_slot(harness):
    """a connection that does not present the job's token (here
    one that sends garbage, one that sends nothing) is dropped without the
    id, and the real rank is still served."""
    import time

    port = free_port()
    p0 = subprocess.Popen([harness], env=clean_env(RANK=0, WORLD_SIZE=2, LIFE_BOOTSTRAP_PORT=port),
                          stdout=subprocess.PIPE, text=True)
    got = []
    for payload in (b"GET / HTTP/1.0\r\n\r\n", None):
        for _ in range(200):  # rank 0 may not be listening yet
            try:
                c = socket.create_connection(("127.0.0.1", port), timeout=5)
                break
            except OSError:
                time.sleep(0.05)
        with c:
            if payload:
                c.sendall(payload)
            c.settimeout(5)
            try:
                got.append(c.recv(256))
            except socket.timeout:
                got.append(b"timeout")
    assert all(g in (b"", b"timeout") or not g.startswith(b"LIFEUID1") for g in got), got
    p1 = subprocess.Popen([harness], env=clean_env(RANK=1, WORLD_SIZE=2, LIFE_BOOTSTRAP_PORT=port),
                          stdout=subprocess.PIPE, text=True)
    outs = [p.communicate(timeout=60)[0] for p in (p0, p1)]
    assert p0.returncode == 0 and p1.returncode == 0, outs
    assert outs[0].split(" id ")[1] == outs[1].split(" id ")[1]


def test_other_job_token_is_refused(harness):
    """Two ranks whose job tokens differ (LIFE_BOOTSTRAP_TOKEN) do not pair:
    rank 1 gets no id and both time out instead of RCCL joining the wrong job."""
    port = free_port()
    procs = [subprocess.Popen([harness], env=clean_env(RANK=r, WORLD_SIZE=2, LIFE_BOOTSTRAP_PORT=port,
                                                         LIFE_BOOTSTRAP_TOKEN=f"job{r}"),
                              stdout=subprocess.PIPE, text=True) for r in (1, 0)]
    outs = [p.communicate(timeout=90)[0] for p in procs]
    assert all(p.returncode == 1 for p in procs), outs


def test_unreachable_rank0_is_bounded(harness):
    """a non-zero rank whose MASTER_ADDR never answers gives up at
    the timeout (non-blocking connect), not after the kernel's SYN retries."""
    import time

    t = time.monotonic()
    r = subprocess.run([harness], env=clean_env(RANK=1, WORLD_SIZE=2, MASTER_ADDR="10.255.255.1",
                                                MASTER_PORT=free_port()),
                       capture_output=True, text=True, timeout=90)
    assert r.returncode == 1 and " rc -1 " in r.stdout, r.stdout
    assert time.monotonic() - t < 40
