"""Compare one libfwav build's fp16 search with its all-f32 kernel on a config (tools only): mismatching rows,
and for a few of them the exact scores of the differing candidates.  usage: python tools/ex_diff.py lib.so"""
import ctypes as C
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "audio-compression_amd")]
import numpy as np
import torch

import __graft_entry__

__graft_entry__.build()
from fwav import engine, synth  # noqa: E402
from fwav._lib import SIGNATURES, call, size_call  # noqa: E402

L = C.CDLL(os.path.abspath(sys.argv[1]))
res_t, args = SIGNATURES["fwav_sim_topk"]
L.fwav_sim_topk.restype, L.fwav_sim_topk.argtypes = res_t, args
L.fwav_sim_topk_workspace_size.restype = C.c_size_t
L.fwav_sim_topk_workspace_size.argtypes = [C.c_int64, C.c_int64, C.c_int]
cfg = os.environ.get("AB_CFG", "cfg3")
sig_h, _, _ = synth.make_config_signal(cfg)
tile = synth.CONFIGS[cfg]["tile"]
sig = torch.from_numpy(sig_h).cuda()
r = engine.compress_device(sig, tile, 64, keep_intermediates=True)
torch.cuda.synchronize()
nd, nr = r.n_domains, r.n_ranges
rs, step = engine.geometry(tile)
st = torch.cuda.current_stream().cuda_stream
emb16 = torch.empty(2 * ((nd + 255) // 256) * 256 * 16, dtype=torch.float16, device="cuda")
tab = engine.embed_tables(rs, torch.device("cuda"))
pool = torch.empty(nd * rs, device="cuda")
emb = torch.empty(nd * 16, device="cuda")
ws = torch.empty(max(size_call("fwav_pool_workspace_size", sig.numel(), tile, rs, step), 16), dtype=torch.uint8,
                 device="cuda")
call("fwav_pool_embed", sig.data_ptr(), sig.numel(), tile, rs, step, tab.data_ptr(), pool.data_ptr(), emb.data_ptr(),
     emb16.data_ptr(), ws.data_ptr(), ws.numel(), st)
nq = int(r.n_active.item())
active = r.active[:nq].clone()
n_active = torch.tensor([nq], dtype=torch.int32, device="cuda")
wsn = L.fwav_sim_topk_workspace_size(nq, nd, 64)
wsk = torch.empty(wsn, dtype=torch.uint8, device="cuda")
outs = []
for e16 in (emb16.data_ptr(), None):
    cand = torch.full((nr * 64,), -7, dtype=torch.int32, device="cuda")
    rc = L.fwav_sim_topk(emb.data_ptr(), e16, nd, active.data_ptr(), n_active.data_ptr(), nq, 0, 64, 16,
                         cand.data_ptr(), None, wsk.data_ptr(), wsn, st)
    torch.cuda.synchronize()
    assert rc == 0
    outs.append(cand.view(nr, 64)[active.long()].cpu().numpy())
    if e16 is not None:
        o = wsn - 4 - 4 * max(nq, 1)
        n_ovf = int(wsk[o:o + 4].view(torch.int32).item())
        ovf = set(wsk[o - 4 * nq:o].view(torch.int32)[:n_ovf].cpu().numpy().tolist())
a, b = outs
bad = np.nonzero((a != b).any(axis=1))[0]
act = active.cpu().numpy()
print(f"{cfg}: active {nq}, overflowed {n_ovf}, mismatching rows {len(bad)} "
      f"({sum(int(act[i]) in ovf for i in bad)} of them overflowed)", flush=True)
E = emb.view(nd, 16).double()
for i in bad[:5]:
    q = int(act[i])
    s = (E * E[q]).sum(-1)
    sa, sb = s[torch.from_numpy(a[i].astype(np.int64)).cuda().clamp(min=0)], s[torch.from_numpy(b[i].astype(np.int64)).cuda()]
    only_a = sorted(set(a[i].tolist()) - set(b[i].tolist()))
    only_b = sorted(set(b[i].tolist()) - set(a[i].tolist()))
    kth = torch.topk(s, 64).values[-1].item()
    print(f" q {q}: f16-only {only_a[:6]} f32-only {only_b[:6]}  min f16 {sa.min().item():.7f} min f32 "
          f"{sb.min().item():.7f} exact K-th {kth:.7f}; first diff at {int(np.argmax(a[i] != b[i]))}", flush=True)
