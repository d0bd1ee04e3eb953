"""Which HIP runtime(s) a process maps when libfwav.so is loaded before / after torch (diagnostic).
usage: python tools/diag/hip_runtime_order.py lib-first|torch-first"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "audio-compression_amd")]


def maps():
    return sorted({l.split()[-1] for l in open("/proc/self/maps") if "amdhip64" in l or "hsa-runtime" in l})


order = sys.argv[1]
if order == "torch-first":
    import torch
    torch.zeros(1, device="cuda")
from fwav import _lib  # noqa: E402
L = _lib.product_lib()
print("after lib load:", maps(), flush=True)
import torch  # noqa: E402
x = torch.arange(4096, dtype=torch.float32, device="cuda")
print("after torch init:", maps(), flush=True)
from fwav import engine  # noqa: E402
sig = torch.randn(44100, device="cuda")
r = engine.compress_device(sig, 2048, 64)
torch.cuda.synchronize()
print(order, "OK", r.n_ranges, flush=True)
