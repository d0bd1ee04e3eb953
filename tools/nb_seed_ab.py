"""Experiment (tools only): band limits seeded from the neighbouring queries' results.  Query i is domain row i
(quirk Q1), so the top K of queries i − 1 and i + 1, shifted by ±1 and widened by s ∈ −2..2, hold K distinct domains
whose exact scores against query i give a valid lower bound on its K-th score (the K-th of the distinct union).  The
seeds are computed on the device with torch from a finished search and fed to an -DFWAV_TOPK_EXTSEED build, for every
query ("all") or for every other one ("odd": what a search that finishes the even queries first could use).
usage: python tools/nb_seed_ab.py tools/ab/libfwav_ext.so [shifts=2]"""
import os as _os_dbg
_os_dbg.environ.setdefault("FWAV_DEBUG_LIBRARY", "1")  # the search knobs: libfwav_debug.so
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
from fwav._lib import SIGNATURES, call  # noqa: E402

L = C.CDLL(os.path.abspath(sys.argv[1]))
SH = int(sys.argv[2]) if len(sys.argv) > 2 else 2
for n in ("fwav_debug_sim_topk", "fwav_sim_topk_workspace_size"):
    getattr(L, n).restype, getattr(L, n).argtypes = SIGNATURES[n]
cfgname = os.environ.get("AB_CFG", "cfg2")
sig = torch.from_numpy(synth.make_config_signal(cfgname, seed=0)[0]).cuda()
K = 64
r = engine.compress_device(sig, 2048, K, keep_intermediates=True, tie_order="index")
torch.cuda.synchronize()
nd, nr = r.n_domains, r.n_ranges
emb16 = torch.empty(2 * ((nd + 255) // 256) * 256 * 16, dtype=torch.float16, device="cuda")
call("fwav_emb16_from_emb", r.emb.data_ptr(), nd, emb16.data_ptr(), torch.cuda.current_stream().cuda_stream)
emb = r.emb
E = emb.view(nd, 16)
st = torch.cuda.current_stream().cuda_stream
nq = int(os.environ.get("AB_NQ", nr))
active = torch.arange(nq, dtype=torch.int32, device="cuda")
n_active = torch.tensor([nq], dtype=torch.int32, device="cuda")
wsn = L.fwav_sim_topk_workspace_size(nq, nd, K)
wsk = torch.empty(wsn, dtype=torch.uint8, device="cuda")
cand = r.cand.view(nr, K).long()
kth_exact = (E[:nr].double() * E[cand[:, K - 1]].double()).sum(1)

# neighbour seeds (exact K-th of the distinct shifted union)
nbseed = torch.full((nr,), -float("inf"), dtype=torch.float64, device="cuda")
shifts = torch.arange(-SH, SH + 1, device="cuda")
for a in range(0, nr, 16384):
    b = min(nr, a + 16384)
    i = torch.arange(a, b, device="cuda")
    parts = []
    for nb, off in ((i - 1, 1), (i + 1, -1)):
        ok = (nb >= 0) & (nb < nr)
        c = cand[nb.clamp(0, nr - 1)] + off                      # [m, K]
        c = (c[:, :, None] + shifts[None, None, :]).reshape(len(i), -1)
        c = torch.where(ok[:, None], c, torch.full_like(c, -1))
        parts.append(c)
    c = torch.cat(parts, 1)
    c = torch.where((c >= 0) & (c < nd), c, torch.full_like(c, -1))
    c, _ = c.sort(1)
    dup = torch.zeros_like(c, dtype=torch.bool)
    dup[:, 1:] = c[:, 1:] == c[:, :-1]
    valid = (c >= 0) & ~dup
    sc = (E[i].double()[:, None, :] * E[c.clamp(0)].double()).sum(2)
    sc = torch.where(valid, sc, torch.full_like(sc, -float("inf")))
    top = sc.topk(K, dim=1).values[:, K - 1]
    nbseed[a:b] = top
gap = (kth_exact - nbseed)[torch.isfinite(nbseed)]
print(f"neighbour seeds s=-{SH}..{SH}: gap to exact K-th mean {gap.mean().item():.4f} median {gap.median().item():.4f}"
      f" p99 {gap.quantile(0.99).item():.4f}; invalid {(gap < 0).sum().item()}", flush=True)
base = (nbseed - 3 * 2.0e-3).float()
ref = None
for name in ("none", "odd", "all", "ideal"):
    if name == "none":
        seeds = torch.full((nr,), -float("inf"), device="cuda")
    elif name == "odd":
        seeds = base.clone()
        seeds[0::2] = -float("inf")
    elif name == "all":
        seeds = base
    else:
        seeds = (kth_exact - 3 * 2.0e-3).float()
    times = []
    for rep in range(4):
        out = torch.empty(nq * K, dtype=torch.int32, device="cuda")
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = L.fwav_debug_sim_topk(emb.data_ptr(), emb16.data_ptr(), nd, active.data_ptr(), n_active.data_ptr(), nq,
                                   0, K, out.data_ptr(), wsk.data_ptr(), wsk.numel(), 0, seeds.data_ptr(), st)
        e1.record()
        torch.cuda.synchronize()
        assert rc == 0
        if rep:
            times.append(e0.elapsed_time(e1))
    if ref is None:
        ref = out.clone()
    print(f"{cfgname} nq={nq} seeds {name:5s}: median {np.median(times):7.2f} ms  identical={bool(torch.equal(out, ref))}",
          flush=True)
