"""Experiment (tools only): would a sampled group-max bound make a good initial band limit?  For a sample of every
F-th 256-domain chunk, the domains are dealt into 64 groups the way a stream wave's lanes see them (lane half,
tile chain, sample-chunk ordinal mod 8); the smallest of the 64 group maxima is a lower bound on the K-th score
(64 distinct domains reach it).  Prints how far the bound is from the exact K-th (mean / quantiles), next to the
exact K-th of the same sample, and times an -DFWAV_TOPK_EXTSEED build seeded with each (the prepass itself not
included).  usage: AB_NQ=... python tools/bound_ab.py tools/ab/libfwav_ext.so F..."""
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
for n in ("fwav_debug_sim_topk", "fwav_sim_topk_workspace_size"):
    getattr(L, n).restype, getattr(L, n).argtypes = SIGNATURES[n]
sig = torch.from_numpy(synth.noise(60.0, 44100)).cuda()
r = engine.compress_device(sig, 2048, 64, keep_intermediates=True)
torch.cuda.synchronize()
nd, nr = r.n_domains, r.n_ranges
emb16 = torch.empty(2 * ((nd + 255) // 256) * 256 * 16, dtype=torch.float16, device="cuda")
tab = engine.embed_tables(8, torch.device("cuda"))
pool = torch.empty(nd * 8, device="cuda")
emb = torch.empty(nd * 16, device="cuda")
ws = torch.empty(16 << 20, dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream().cuda_stream
call("fwav_pool_embed", sig.data_ptr(), sig.numel(), 2048, 8, 2, tab.data_ptr(), pool.data_ptr(), emb.data_ptr(),
     emb16.data_ptr(), ws.data_ptr(), ws.numel(), st)
nq = int(os.environ.get("AB_NQ", nr))
active = torch.arange(nq, dtype=torch.int32, device="cuda")
n_active = torch.tensor([nq], dtype=torch.int32, device="cuda")
wsn = L.fwav_sim_topk_workspace_size(nq, nd, 64)
wsk = torch.empty(wsn, dtype=torch.uint8, device="cuda")
E = emb.view(nd, 16)
d16 = 2.0e-3
kth = r.cand.view(nr, 64)[:nq, 63].long()
exact_k = (E[:nq].double() * E[kth].double()).sum(1)


def timed(seeds):
    times = []
    for rep in range(4):
        cand = torch.empty(nq * 64, dtype=torch.int32, device="cuda")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = L.fwav_debug_sim_topk(emb.data_ptr(), emb16.data_ptr(), nd, active.data_ptr(), n_active.data_ptr(), nq, 0,
                                   64, cand.data_ptr(), wsk.data_ptr(), wsk.numel(), 0, seeds.data_ptr(), st)
        e1.record()
        torch.cuda.synchronize()
        assert rc == 0
        if rep:
            times.append(e0.elapsed_time(e1))
    return float(np.median(times)), cand


def gap_text(b):
    g = (exact_k - b.double()).cpu().numpy()
    return f"gap mean {g.mean():.4f} p10 {np.quantile(g, 0.1):.4f} p50 {np.median(g):.4f} p90 {np.quantile(g, 0.9):.4f}"


t0, ref = timed(torch.full((nq,), -float("inf"), device="cuda"))
print(f"no external seed: {t0:.2f} ms", flush=True)
ti, _ = timed((exact_k - 3 * d16).float())
print(f"ideal (exact K-th - 3δ): {ti:.2f} ms", flush=True)
nch = (nd + 255) // 256
for F in [int(x) for x in sys.argv[2:]]:
    chunks = torch.arange(0, nch, F, device="cuda")
    dom = (chunks[:, None] * 256 + torch.arange(256, device="cuda")[None, :]).reshape(-1)
    ordinal = torch.arange(len(chunks), device="cuda")[:, None].expand(-1, 256).reshape(-1)
    ok = dom < nd
    dom, ordinal = dom[ok], ordinal[ok]
    row = dom & 31
    grp = ((ordinal & 7) * 4 + ((dom >> 5) & 3)) * 2 + ((row >> 2) & 1)
    Es = E[dom]
    bound = torch.empty(nq, dtype=torch.float64, device="cuda")
    samp_k = torch.empty(nq, dtype=torch.float64, device="cuda")
    for a in range(0, nq, 2048):
        b = min(a + 2048, nq)
        sc = E[a:b] @ Es.T  # f32 scores (the kernel's s16 is within δ of these)
        gm = torch.full((b - a, 64), -float("inf"), device="cuda").scatter_reduce(
            1, grp[None, :].expand(b - a, -1), sc, reduce="amax")
        bound[a:b] = gm.min(1).values.double()
        samp_k[a:b] = sc.topk(64, dim=1).values[:, -1].double()
    tb, cb = timed((bound - 3 * d16).float())
    ts, cs = timed((samp_k - 3 * d16).float())
    print(f"F={F:3d} ({len(dom)} domains): group-max bound {gap_text(bound)} -> {tb:.2f} ms  same={bool(torch.equal(cb, ref))}",
          flush=True)
    print(f"       sample K-th {gap_text(samp_k)} -> {ts:.2f} ms  same={bool(torch.equal(cs, ref))}", flush=True)
