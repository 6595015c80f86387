"""Diagnostic (GPU box): does libsr_amd's HIP context come up when torch touched the GPU first?
usage: python tools/order_probe.py {lib_first,torch_first,torch_import_only}"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "symbolicregression.jl_amd")]
mode = sys.argv[1]
import sr_amd
if mode == "lib_first":
    ctx = sr_amd.get_context(0)
    import torch
    torch.cuda.set_device(0)
    t = torch.ones(4, device="cuda"); print("torch ok", float(t.sum()))
elif mode == "torch_first":
    import torch
    torch.cuda.set_device(0)
    t = torch.ones(4, device="cuda"); print("torch ok", float(t.sum()))
    ctx = sr_amd.get_context(0)
else:
    import torch
    ctx = sr_amd.get_context(0)
print(mode, "context ok")
maps = open("/proc/self/maps").read()
print(sorted({l.split()[-1] for l in maps.splitlines() if "amdhip64" in l or "hsa-runtime" in l}))
