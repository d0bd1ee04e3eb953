"""Diagnostic: how many rows the search lists with exact score ties at cfg2 / cfg3 (in-set vs K-th place), how many
fwav_tie_check sends to the host, what the ties stage costs, and a few example rows (scores around the K-th).
usage: python tools/diag/tie_stats.py cfg2 [cfg3 ...]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "audio-compression_amd")]
import numpy as np
import torch

from fwav import engine, synth, ties
from fwav._lib import call

dev = torch.device("cuda", 0)
for name in sys.argv[1:]:
    cfg = synth.CONFIGS[name]
    sig_h, _, _ = synth.make_config_signal(name, seed=0)
    sig = torch.from_numpy(sig_h).to(dev)
    tile, K = cfg["tile"], cfg["top_k"]
    for order in ("index", "numpy", "numpy"):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev = {}
        r = engine.compress_device(sig, tile, K, energy_thresh=1e-4, keep_intermediates=True, tie_order=order,
                                   events=ev)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) * 1e3
        st = {k: v[0].elapsed_time(v[1]) for k, v in ev.items()}
        print(f"{name} {order}: {dt:.1f} ms wall, stages {({k: round(v, 3) for k, v in st.items()})}, "
              f"n_ties {r.n_ties} n_resolved {r.n_resolved}", flush=True)
    # the ties list itself (index order run): boundary vs in-set
    m = r.n_ranges
    nd = r.n_domains
    tl = torch.empty(engine.size_call("fwav_tie_list_size", m), dtype=torch.int32, device=dev)
    wk = engine.size_call("fwav_sim_topk_workspace_size", m, nd, K)
    wsk = torch.empty(wk, dtype=torch.uint8, device=dev)
    cand = torch.empty(m * K, dtype=torch.int32, device=dev)
    emb16 = torch.empty(2 * ((nd + 255) // 256) * 256 * 16, dtype=torch.float16, device=dev)
    # rebuild the fp16 table (compress_device does not keep it)
    rs, step = engine.geometry(tile)
    tab = engine.embed_tables(rs, dev)
    pool = torch.empty(nd * rs, dtype=torch.float32, device=dev)
    emb = torch.empty(nd * 16, dtype=torch.float32, device=dev)
    wsp_n = engine.size_call("fwav_pool_workspace_size", sig.numel(), tile, rs, step)
    wsp = torch.empty(max(wsp_n, 16), dtype=torch.uint8, device=dev)
    st_ = torch.cuda.current_stream().cuda_stream
    call("fwav_pool_embed", sig.data_ptr(), sig.numel(), tile, rs, step, tab.data_ptr(), pool.data_ptr(),
         emb.data_ptr(), emb16.data_ptr(), wsp.data_ptr(), wsp_n, st_)
    act = r.active
    call("fwav_sim_topk", emb.data_ptr(), emb16.data_ptr(), nd, act.data_ptr(), r.n_active.data_ptr(), m, 0, K,
         ties.blas_threads(), cand.data_ptr(), tl.data_ptr(), wsk.data_ptr(), wk, st_)
    torch.cuda.synchronize()
    n = int(tl[0])
    ent = tl[1:1 + 9 * n].view(-1, 9)[:, 0].cpu().numpy()  # records of 9 int32 (fwav.h)
    print(f"  listed {n}: K-th-place ties {(ent & 1).sum()}, in-set only {(~ent & 1).sum()}", flush=True)
    embh = emb.view(-1, 16)
    for e in ent[:6]:
        q = int(e >> 1)
        sc = (embh @ embh[q]).cpu().numpy()  # torch order, only for a look at the neighbourhood of the K-th
        srt = np.sort(sc)[::-1]
        c = cand.view(-1, K)[q].cpu().numpy()
        print(f"   row {q} boundary {e & 1}: top K+2 (approx) {srt[K - 3:K + 2].tolist()}; "
              f"cand scores at K-2..K {sc[c[K - 3:]].tolist()}", flush=True)
