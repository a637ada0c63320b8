"""Probe: does loading liblife_mi355x.so next to torch's bundled HIP runtime
survive process exit?  mode: lib_only | lib_then_torch | torch_then_lib | torch_cuda"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-and-open-mp_amd"))
mode = sys.argv[1]
if mode in ("torch_then_lib",):
    import torch
import life_mi355x as lm
lm._lib()
if mode in ("lib_then_torch", "torch_cuda"):
    import torch
if mode == "torch_cuda":
    torch.cuda.set_device(0); torch.cuda.synchronize()
life = lm.Life(4096, 4096, kernel="bit"); life.fill_random(1); life.step(10); print("live", life.live_count()); life.close()
if mode == "torch_cuda":
    torch.cuda.synchronize()
print("ok", mode, flush=True)
