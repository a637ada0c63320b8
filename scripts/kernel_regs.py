#!/usr/bin/env python3
"""VGPR / spill counts of the kernels in a hipcc object (measurement tool):
extracts the gfx950 code object from the object's .hip_fatbin section and
prints name, vgpr_count, vgpr_spill_count for kernels matching a pattern.

  python3 scripts/kernel_regs.py mpi-and-open-mp_amd/build/life_kernels.hip.o tstep_bit tflow
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def main():
    obj, pats = sys.argv[1], sys.argv[2:] or [""]
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "k.co")
        subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fat}", obj], check=True)
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={fat}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout
    cur, rows = {}, []
    for ln in notes.splitlines():
        ln = ln.strip()
        m = re.match(r"\.(name|vgpr_count|vgpr_spill_count|sgpr_spill_count|agpr_count):\s+(\S+)", ln)
        if not m:
            continue
        if m.group(1) == "name":
            if cur:
                rows.append(cur)
            cur = {"name": m.group(2)}
        else:
            cur[m.group(1)] = m.group(2)
    rows.append(cur)
    names = [r.get("name", "") for r in rows]
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True).stdout.splitlines()
    for r, dn in zip(rows, dem):
        if any(p in dn for p in pats):
            print(f"{dn[:110]:110s} vgpr {r.get('vgpr_count')} spill {r.get('vgpr_spill_count')}")


if __name__ == "__main__":
    main()
