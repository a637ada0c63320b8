"""Static guards on the shipped gfx950 code object (CPU only, no GPU).

The bit tile's generation loop is VALU-bound; how early the compiler issues
each row's two ds_bpermute ahead of their first use decides whether the LDS
latency hides behind other VALU work.  A source change that looked unrelated
(the deep-halo store predicate, evaluated after the loop) once moved them next
to their s_waitcnt (mean 7.7 -> 1.7 instructions apart) and cost 8 % of the
driver-shaped call on the same box (profiles/r04/e: 0.417-0.430 -> 0.450-0.461
ms per launch).  These tests disassemble the built object and pin the
schedule's shape, the VGPR budget (3 tiles per CU need <= 80) and the
instruction counts DESIGN.md §5.1 models (22 VALU per pair row: 20 v_bitop3 +
2 v_alignbit, 2 ds_bpermute).  (VGPR banks are not pinned: a build with 155
v_bitop3 reading three sources from one bank ran as fast as one with 11,
profiles/r04/i.)
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(ROOT, "mpi-and-open-mp_amd", "build", "life_kernels.hip.o")
LLVM = "/opt/rocm/lib/llvm/bin"
KERNEL = "tstep_bit_kernel<24, true, true, 8>"  # the 65536^2 single-GPU instance


@pytest.fixture(scope="module")
def isa(tmp_path_factory):
    if not os.path.exists(OBJ) or not os.path.exists(f"{LLVM}/llvm-objdump"):
        pytest.skip("built object or llvm-objdump missing")
    d = tmp_path_factory.mktemp("isa")
    fat, co = str(d / "fat.bin"), str(d / "k.co")
    subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fat}", OBJ], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    dis = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", co], capture_output=True, text=True,
                         check=True).stdout
    dis = subprocess.run(["c++filt"], input=dis, capture_output=True, text=True).stdout
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
    return dis, notes


def kernel_lines(dis, kernel=KERNEL):
    """(address, op, text) of every instruction of `kernel`."""
    lines = dis.splitlines()
    start = next(i for i, ln in enumerate(lines) if re.match(r"^[0-9a-f]+ <", ln) and kernel in ln)
    end = next(i for i in range(start + 1, len(lines)) if re.match(r"^[0-9a-f]+ <.*>:$", lines[i]))
    out = []
    for ln in lines[start + 1:end]:
        m = re.search(r"//\s*([0-9A-Fa-f]+):", ln)
        text = ln.split("//")[0].strip()
        if m and text:
            out.append((int(m.group(1), 16), text.split()[0], text))
    return out


def generation_loops(lines):
    """Op sequences of the kernel's generation loops with a full-height
    window: the body of every backward branch whose loop holds a barrier and
    480 v_bitop3 (24 pair rows x 20)."""
    out = []
    for k, (addr, op, text) in enumerate(lines):
        m = re.match(r"s_cbranch_\w+ (\d+)$", text)
        if not m:
            continue
        simm = int(m.group(1))
        if simm < 0x8000:
            continue  # forward
        target = addr + 4 + 4 * (simm - 0x10000)
        ops = [o for a, o, _ in lines if target <= a <= addr]
        if "s_barrier" in ops and ops.count("v_bitop3_b32") == 480:
            out.append(ops)
    return out


def test_generation_loop_counts(isa):
    loops = generation_loops(kernel_lines(isa[0]))
    assert loops, "no full-height generation loop found"
    for ops in loops:  # 24 pair rows x (20 v_bitop3 + 2 v_alignbit + 2 ds_bpermute), one barrier
        assert ops.count("v_alignbit_b32") == 48 and ops.count("ds_bpermute_b32") == 48
        assert ops.count("s_barrier") == 1


def test_bpermute_issued_ahead_of_use(isa):
    for ops in generation_loops(kernel_lines(isa[0])):
        gaps = []
        for i, o in enumerate(ops):
            if o == "ds_bpermute_b32":
                gaps.append(next(k for k in range(i, len(ops)) if ops[k] == "s_waitcnt") - i)
        assert sum(gaps) / len(gaps) >= 5.0, f"ds_bpermute -> s_waitcnt mean {sum(gaps) / len(gaps):.2f}"


def test_vgpr_budget(isa):
    notes = isa[1]
    names = re.findall(r"\.name:\s+(\S+)", notes)
    vgprs = re.findall(r"\.vgpr_count:\s+(\d+)", notes)
    spills = re.findall(r"\.vgpr_spill_count:\s+(\d+)", notes)
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
    found = [(int(v), int(s)) for n, v, s in zip(dem, vgprs, spills) if KERNEL in n]
    assert found and all(v <= 80 and s == 0 for v, s in found), found


BYTE_KERNEL = "tstep_byte_kernel<48, 32, true, true, 8>"  # the 65536^2 byte instance


def test_byte_permutes_issued_ahead(isa):
    """The byte tile's generation loop keeps its left-neighbour permutes two
    rows ahead of their use (LIFE_BYTE_BP_AHEAD = 2, rows fenced in order;
    -2 % per launch, profiles/r04/byte_ab): its waits allow two younger LDS
    operations in flight.  Unfenced, the compiler waits for every permute
    right after issuing it (lgkmcnt(0) only)."""
    lines = kernel_lines(isa[0], BYTE_KERNEL)
    loops = []
    for addr, op, text in lines:
        m = re.match(r"s_cbranch_\w+ (\d+)$", text)
        if not m or int(m.group(1)) < 0x8000:
            continue
        target = addr + 4 + 4 * (int(m.group(1)) - 0x10000)
        body = [t for a, _, t in lines if target <= a <= addr]
        if any(t.startswith("s_barrier") for t in body) and len(body) > 300:
            loops.append(body)
    assert loops, "no byte generation loop found"
    for body in loops:
        ahead = sum(1 for t in body if t == "s_waitcnt lgkmcnt(2)")
        assert ahead >= 40, f"{ahead} waits with two permutes in flight"


FLOW_KERNEL = "tflow_kernel<24, true, true, 1, 8, false>"  # the dataflow form (write-through hand-off)


def test_flow_permutes_issued_ahead(isa):
    """The dataflow tiles' generation loop issues each row's two permutes one
    row ahead (LIFE_FLOW_BP_AHEAD = 1): its waits leave the next row's two
    (and the current row's second) in flight -- lgkmcnt(2) / (3).  Left to
    the compiler, every permute sat right before its wait there (mean
    distance 1.8 instructions against 7.6-9.8 in the per-launch tiles)."""
    lines = kernel_lines(isa[0], FLOW_KERNEL)
    loops = []
    for addr, op, text in lines:
        m = re.match(r"s_cbranch_\w+ (\d+)$", text)
        if not m or int(m.group(1)) < 0x8000:
            continue
        target = addr + 4 + 4 * (int(m.group(1)) - 0x10000)
        body = [t for a, _, t in lines if target <= a <= addr]
        ops = [t.split()[0] for t in body]
        if "s_barrier" in ops and ops.count("v_bitop3_b32") == 480:
            loops.append(body)
    assert loops, "no dataflow generation loop found"
    for body in loops:
        ahead = sum(1 for t in body if t in ("s_waitcnt lgkmcnt(2)", "s_waitcnt lgkmcnt(3)"))
        assert ahead >= 40, f"{ahead} waits with permutes of the next row in flight"
