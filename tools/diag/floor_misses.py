"""Diagnostic: the floor's miss counts and per-pass times for the cfg2 search called with the engine's own active list
(fwav_prune's order) against arange(n).  usage: python tools/diag/floor_misses.py"""
import os
import struct
import sys

os.environ.setdefault("FWAV_DEBUG_LIBRARY", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "audio-compression_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import __graft_entry__  # noqa: E402

__graft_entry__.build()
from fwav import engine, synth  # noqa: E402
from fwav._lib import call, size_call  # noqa: E402

sig = torch.from_numpy(synth.make_config_signal("cfg2")[0]).cuda()
r = engine.compress_device(sig, 2048, 64, energy_thresh=1e-4, keep_intermediates=True)
torch.cuda.synchronize()
nd, nr = r.n_domains, r.n_ranges
na = int(r.n_active.item())
act_engine = r.active[:na].clone()
print("n_active", na, "sorted:", bool((act_engine[1:] > act_engine[:-1]).all().item()),
      "first", act_engine[:8].tolist(), flush=True)
st = torch.cuda.current_stream().cuda_stream
emb16 = torch.empty(2 * ((nd + 255) // 256) * 256 * 16, dtype=torch.float16, device="cuda")
call("fwav_emb16_from_emb", r.emb.data_ptr(), nd, emb16.data_ptr(), st)
PIL = 4 * (1024 * 512 * 8 + 512)
for name, act in (("engine order", act_engine), ("arange", torch.arange(na, dtype=torch.int32, device="cuda"))):
    n_act = torch.tensor([na], dtype=torch.int32, device="cuda")
    wsn = size_call("fwav_sim_topk_workspace_size", nr, nd, 64)
    ws = torch.zeros(wsn, dtype=torch.uint8, device="cuda")
    ts = []
    for rep in range(5):
        cand = torch.empty(nr * 64, dtype=torch.int32, device="cuda")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        call("fwav_sim_topk", r.emb.data_ptr(), emb16.data_ptr(), nd, act.data_ptr(), n_act.data_ptr(), nr, 0, 64, 1,
             cand.data_ptr(), None, ws.data_ptr(), wsn, st)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    b = ws[wsn - PIL - 8 - 4 * (nr + 1) - 4:wsn - PIL].cpu().numpy().tobytes()
    n1 = struct.unpack("<i", b[:4])[0]
    n2, k0, k1 = struct.unpack("<iII", b[-12:])
    f = lambda k: struct.unpack("<f", struct.pack("<I", (k & 0x7FFFFFFF) if k & 0x80000000 else (~k & 0xFFFFFFFF)))[0]
    print(f"{name}: median {np.median(ts[1:]):.3f} ms; floor {f(k0):.4f}, second floor {f(k1):.4f}; "
          f"{n1} to the second pass, {n2} to the third", flush=True)
