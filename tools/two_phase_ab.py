"""Experiment (tools only): the two-launch strided search of DESIGN §10 item 6.  Launch 1 searches every S-th query
(no external seeds); launch 2 searches the rest, each seeded with the exact K-th best score of the distinct union of
its nearest finished neighbours' candidate rows, shifted by the distance and widened by ±SH (query i is domain row i,
Q1), minus 3δ — a valid lower bound, fed through an -DFWAV_TOPK_EXTSEED build.  Times launch 1, the seed step (torch
here; a kernel in a product) and launch 2 separately against the single launch, and checks identical candidates.
usage: python tools/two_phase_ab.py tools/ab/libfwav_ext.so [strides=2,4,8] (AB_NQ: first nq queries)"""
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
STRIDES = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "2,4,8").split(",")]
SH = int(os.environ.get("AB_SHIFTS", 2))
for n in ("fwav_debug_sim_topk", "fwav_sim_topk_workspace_size"):
    getattr(L, n).restype, getattr(L, n).argtypes = SIGNATURES[n]
cfgname = os.environ.get("AB_CFG", "cfg2")
cfg = synth.CONFIGS[cfgname]
K = cfg["top_k"]
sig = torch.from_numpy(synth.make_config_signal(cfgname, seed=0)[0]).cuda()
r = engine.compress_device(sig, cfg["tile"], K, keep_intermediates=True, tie_order="index")
torch.cuda.synchronize()
nd, nr = r.n_domains, r.n_ranges
emb16 = torch.empty(2 * ((nd + 255) // 256) * 256 * 16, dtype=torch.float16, device="cuda")
st = torch.cuda.current_stream().cuda_stream
call("fwav_emb16_from_emb", r.emb.data_ptr(), nd, emb16.data_ptr(), st)
emb = r.emb
E = emb.view(nd, 16)
nq = int(os.environ.get("AB_NQ", nr))
sizes = [nq] + [len(range(0, nq, s)) for s in STRIDES] + [nq - len(range(0, nq, s)) for s in STRIDES]
wsn = max(L.fwav_sim_topk_workspace_size(m, nd, K) for m in sizes)
wsk = torch.empty(wsn, dtype=torch.uint8, device="cuda")
NEG = torch.full((nq,), -float("inf"), device="cuda")


def search(active, seeds, out):
    m = active.numel()
    na = torch.tensor([m], dtype=torch.int32, device="cuda")
    rc = L.fwav_debug_sim_topk(emb.data_ptr(), emb16.data_ptr(), nd, active.data_ptr(), na.data_ptr(), m, 0, K,
                               out.data_ptr(), wsk.data_ptr(), wsk.numel(), 0, seeds.data_ptr(), st)
    assert rc == 0


def nb_seeds(qb, qa_lo, qa_hi, cand):
    """Seeds for queries qb from their finished neighbours qa_lo ≤ qb ≤ qa_hi (−1: none)."""
    out = torch.empty(qb.numel(), dtype=torch.float32, device="cuda")
    shifts = torch.arange(-SH, SH + 1, device="cuda")
    cv = cand.view(-1, K).long()
    for a in range(0, qb.numel(), 16384):
        i = qb[a:a + 16384].long()
        parts = []
        for nb in (qa_lo[a:a + 16384].long(), qa_hi[a:a + 16384].long()):
            ok = nb >= 0
            c = cv[nb.clamp(0)] + (i - nb)[:, None]
            c = (c[:, :, None] + shifts[None, None, :]).reshape(len(i), -1)
            parts.append(torch.where(ok[:, None], c, torch.full_like(c, -1)))
        c = torch.cat(parts, 1)
        c = torch.where((c >= 0) & (c < nd), c, torch.full_like(c, -1))
        c, _ = c.sort(1)
        dup = torch.zeros_like(c, dtype=torch.bool)
        dup[:, 1:] = c[:, 1:] == c[:, :-1]
        valid = (c >= 0) & ~dup
        sc = (E[i].double()[:, None, :] * E[c.clamp(0)].double()).sum(2)
        sc = torch.where(valid, sc, torch.full_like(sc, -float("inf")))
        out[a:a + 16384] = (sc.topk(K, dim=1).values[:, K - 1] - 3 * 2.0e-3).float()
    return out


def ev():
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    return e


allq = torch.arange(nq, dtype=torch.int32, device="cuda")
ref = torch.empty(nq * K, dtype=torch.int32, device="cuda")
t = []
for rep in range(5):
    e0 = ev()
    search(allq, NEG, ref)
    e1 = ev()
    torch.cuda.synchronize()
    if rep:
        t.append(e0.elapsed_time(e1))
print(f"{cfgname} nq={nq} K={K} single launch: median {np.median(t):7.2f} ms", flush=True)
for S in STRIDES:
    qa = torch.arange(0, nq, S, dtype=torch.int32, device="cuda")
    mask = torch.ones(nq, dtype=torch.bool, device="cuda")
    mask[qa.long()] = False
    qb = torch.nonzero(mask).flatten().to(torch.int32)
    lo = (qb // S) * S
    hi = lo + S
    hi = torch.where(hi < nq, hi, torch.full_like(hi, -1))
    t1, t2, t3 = [], [], []
    for rep in range(5):
        out = torch.empty(nq * K, dtype=torch.int32, device="cuda")
        e0 = ev()
        search(qa, NEG, out)
        e1 = ev()
        seeds = nb_seeds(qb, lo, hi, out)
        e2 = ev()
        search(qb, seeds, out)
        e3 = ev()
        torch.cuda.synchronize()
        if rep:
            t1.append(e0.elapsed_time(e1))
            t2.append(e1.elapsed_time(e2))
            t3.append(e2.elapsed_time(e3))
    kth = (E[qb.long()].double() * E[out.view(-1, K)[qb.long(), K - 1].long()].double()).sum(1)
    gap = kth - (seeds.double() + 3 * 2.0e-3)
    print(f"{cfgname} nq={nq} stride {S}: launch 1 {np.median(t1):6.2f} ms + seeds {np.median(t2):6.2f} (torch) + "
          f"launch 2 {np.median(t3):6.2f} = search {np.median(t1) + np.median(t3):6.2f} ms; seed gap mean "
          f"{gap.mean().item():.4f} invalid {(gap < 0).sum().item()}; identical={bool(torch.equal(out, ref))}",
          flush=True)
