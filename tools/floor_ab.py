"""Experiment (tools only): a global speculative band floor.  Every query's band limit starts at max(its own seed, τ)
for a constant τ (an -DFWAV_TOPK_EXTSEED build); prints the search time per τ and whether the candidates still equal
the unseeded search's (they do whenever τ is below every query's K-th score − 2δ).
usage: python tools/floor_ab.py tools/ab/libfwav_ext.so 1.70,1.80,1.85"""
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
from fwav._lib import SIGNATURES, call, size_call  # noqa: E402

L = C.CDLL(os.path.abspath(sys.argv[1]))
for n in ("fwav_debug_sim_topk", "fwav_sim_topk_workspace_size"):
    getattr(L, n).restype, getattr(L, n).argtypes = SIGNATURES[n]
sig = torch.from_numpy(synth.make_config_signal("cfg2")[0]).cuda()
r = engine.compress_device(sig, 2048, 64, keep_intermediates=True)
torch.cuda.synchronize()
nd, nr = r.n_domains, r.n_ranges
emb16 = torch.empty(2 * ((nd + 255) // 256) * 256 * 16, dtype=torch.float16, device="cuda")
tab = engine.embed_tables(8, torch.device("cuda"))
pool = torch.empty(nd * 8, device="cuda")
emb = torch.empty(nd * 16, device="cuda")
ws = torch.empty(max(size_call("fwav_pool_workspace_size", sig.numel(), 2048, 8, 2), 16), dtype=torch.uint8,
                 device="cuda")
st = torch.cuda.current_stream().cuda_stream
call("fwav_pool_embed", sig.data_ptr(), sig.numel(), 2048, 8, 2, tab.data_ptr(), pool.data_ptr(), emb.data_ptr(),
     emb16.data_ptr(), ws.data_ptr(), ws.numel(), st)
nq = int(os.environ.get("AB_NQ", nr))
active = torch.arange(nq, dtype=torch.int32, device="cuda")
n_active = torch.tensor([nq], dtype=torch.int32, device="cuda")
wsk = torch.empty(L.fwav_sim_topk_workspace_size(nq, nd, 64), dtype=torch.uint8, device="cuda")
E = emb.view(nd, 16)


def run(seeds):
    cand = torch.empty(nq * 64, dtype=torch.int32, device="cuda")
    ts = []
    for rep in range(4):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = L.fwav_debug_sim_topk(emb.data_ptr(), emb16.data_ptr(), nd, active.data_ptr(), n_active.data_ptr(), nq, 0,
                                   64, cand.data_ptr(), wsk.data_ptr(), wsk.numel(), 0,
                                   seeds.data_ptr() if seeds is not None else None, st)
        e1.record()
        torch.cuda.synchronize()
        assert rc == 0
        if rep:
            ts.append(e0.elapsed_time(e1))
    return float(np.median(ts)), cand


t0, ref = run(None)
kth = (E[:nq].double() * E[ref.view(nq, 64)[:, 63].long()].double()).sum(1)
print(f"no floor: {t0:.2f} ms; exact K-th over the queries: min {kth.min().item():.4f} "
      f"q0.001 {kth.quantile(0.001).item():.4f} median {kth.median().item():.4f}", flush=True)
for tau in [float(x) for x in sys.argv[2].split(",")]:
    t, c = run(torch.full((nq,), tau, device="cuda"))
    print(f"floor {tau:.3f}: {t:.2f} ms  identical={bool(torch.equal(c, ref))}  "
          f"queries below floor+2δ {int((kth < tau + 4e-3).sum())}", flush=True)
