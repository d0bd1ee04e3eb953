"""Experiment (tools only): how much would a tighter initial band limit help?  Seeds every query with the K-th best
exact score over a sample of S domains (minus 3δ, a valid s16 lower bound) computed on the host side with torch, and
times an -DFWAV_TOPK_EXTSEED build with and without them.  usage: python tools/seed_ab.py tools/ab/libfwav_ext.so S..."""
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
from fwav._lib import DEBUG_SIGNATURES, SIGNATURES, call  # noqa: E402

L = C.CDLL(os.path.abspath(sys.argv[1]))
for n in ("fwav_debug_sim_topk", "fwav_sim_topk_workspace_size"):
    getattr(L, n).restype, getattr(L, n).argtypes = {**SIGNATURES, **DEBUG_SIGNATURES}[n]
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
nq = int(os.environ.get("AB_NQ", nr))  # the first nq ranges (one rank's share at N > 1)
active = torch.arange(nq, dtype=torch.int32, device="cuda")
n_active = torch.tensor([nq], dtype=torch.int32, device="cuda")
wsn = L.fwav_sim_topk_workspace_size(nq, nd, 64)
wsk = torch.empty(wsn, dtype=torch.uint8, device="cuda")
E = emb.view(nd, 16)
ref = None
for S in [0] + [int(x) for x in sys.argv[2:]]:
    seeds = torch.full((nr,), -float("inf"), device="cuda")
    if -1000 <= S < 0:  # ideal: the exact K-th best score of every query (from the search's own candidates), minus 3δ
        # (S = -1), or minus (-S)/1000 more (S = -20: 0.020 below the ideal seed)
        kth = r.cand.view(nr, 64)[:, 63].long()
        seeds = ((E[:nr].double() * E[kth].double()).sum(1) - 3 * 2.0e-3 - (0 if S == -1 else -S / 1000.0)).float()
    if S < -1000:
        # one global seed g = (-S - 1000) / 1000 (e.g. -2870: 1.870), capped per query at its ideal seed so that it
        # stays a valid lower bound: the time a global seed would take if its misses were free
        kth = r.cand.view(nr, 64)[:, 63].long()
        ideal = ((E[:nr].double() * E[kth].double()).sum(1) - 3 * 2.0e-3).float()
        seeds = torch.clamp(ideal, max=(-S - 1000) / 1000.0)
        print(f"global seed {(-S - 1000) / 1000.0:.3f}: {(ideal < (-S - 1000) / 1000.0).float().mean().item():.4%} "
              "of the queries below it", flush=True)
    elif S > 0:
        samp = torch.linspace(0, nd - 1, S, device="cuda").long()
        Es = E[samp].double()
        for a in range(0, nr, 32768):
            sc = E[a:min(a + 32768, nr)].double() @ Es.T
            seeds[a:a + 32768] = (sc.topk(64, dim=1).values[:, -1] - 3 * 2.5e-3).float()
    times = []
    for rep in range(4):
        cand = torch.empty(nr * 64, dtype=torch.int32, device="cuda")
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = L.fwav_debug_sim_topk(emb.data_ptr(), emb16.data_ptr(), nd, active.data_ptr(), n_active.data_ptr(), nq, 0,
                                   64, cand.data_ptr(), wsk.data_ptr(), wsk.numel(), int(os.environ.get("AB_DBG", "0")),
                                   seeds.data_ptr(), st)
        e1.record()
        torch.cuda.synchronize()
        assert rc == 0
        if rep:
            times.append(e0.elapsed_time(e1))
    cand = cand[:nq * 64]
    if ref is None:
        ref = cand.clone()
    print(f"sample {S:6d} (-1 = ideal): median {np.median(times):7.2f} ms  seed mean {seeds[seeds > -1e30].mean().item() if S else float('nan'):.4f}"
          f"  identical={bool(torch.equal(cand, ref))}", flush=True)
