#!/usr/bin/env python3
"""What k_merge_pieces reads at cfg2 (diagnostic for VERDICT r5 #3): after one product fwav_sim_topk call, the pieces'
band headers and entries of the split blocks whose key regions the floor's second pass did not reuse, and per query
  n  = the pieces' band entries (the headers' counts: what the merge loads),
  m  = those above Lk (≈ the query's shared limit: the largest piece limit, each piece's own K-th key − 2δ),
  mb = those above the union's K-th key − 2δ (what the merge rescores and sorts).
usage: python tools/diag/merge_inputs.py [--config cfg2]"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "audio-compression_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

K = 64
DELTA = 2.0e-3


def key2f(k):
    k = k.astype(np.uint32)
    pos = (k & 0x80000000) != 0
    bits = np.where(pos, k & 0x7FFFFFFF, ~k)
    return bits.astype(np.uint32).view(np.float32)


def f2key(x):
    b = np.asarray(x, np.float32).view(np.uint32)
    return np.where(b & 0x80000000, ~b, b | 0x80000000).astype(np.uint32)


def kth_12(hi, valid):
    """The greedy select of the kernels: the largest T with its low 12 bits clear and count(hi >= T) >= K (0: < K)."""
    h = np.where(valid, hi, 0).astype(np.int64)
    srt = -np.sort(-h, axis=-1)
    t = srt[..., K - 1]
    return np.where(valid.sum(-1) >= K, t & ~0xFFF, 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    a = ap.parse_args()
    import __graft_entry__
    __graft_entry__.build()
    from fwav import engine, synth
    from fwav._lib import call, size_call, debug_lib
    dev = torch.device("cuda", 0)
    cfg = synth.CONFIGS[a.config]
    sig_h, _, _ = synth.make_config_signal(a.config, seed=0)
    sig = torch.from_numpy(sig_h).to(dev)
    tile = cfg["tile"]
    res = engine.compress_device(sig, tile, K, keep_intermediates=True)
    torch.cuda.synchronize()
    nd, rs, step = res.n_domains, res.range_size, res.domain_step
    n = sig.numel()
    tab = engine.embed_tables(rs, dev)
    pool = torch.empty(nd * rs, dtype=torch.float32, device=dev)
    emb = torch.empty(nd * 16, dtype=torch.float32, device=dev)
    emb16 = torch.empty(2 * ((nd + 255) // 256) * 256 * 16, dtype=torch.float16, device=dev)
    wsp_n = size_call("fwav_pool_workspace_size", n, tile, rs, step)
    wsp = torch.empty(max(wsp_n, 16), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    call("fwav_pool_embed", sig.data_ptr(), n, tile, rs, step, tab.data_ptr(), pool.data_ptr(), emb.data_ptr(),
         emb16.data_ptr(), wsp.data_ptr(), wsp_n, st)
    m = res.n_ranges
    wk = size_call("fwav_sim_topk_workspace_size", m, nd, K)
    wsk = torch.zeros(wk, dtype=torch.uint8, device=dev)
    cand = torch.empty(m * K, dtype=torch.int32, device=dev)
    from fwav import ties
    call("fwav_sim_topk", emb.data_ptr(), emb16.data_ptr(), nd, res.active.data_ptr(), res.n_active.data_ptr(), m, 0,
         K, ties.blas_threads(), cand.data_ptr(), 0, wsk.data_ptr(), wk, st)
    torch.cuda.synchronize()
    # equal to the product's rows except those numpy re-ranked (exact ties, fwav.ties)
    same = (cand.view(-1, K) == res.cand.view(-1, K)).all(1)
    if res.resolved is not None and res.resolved.numel():
        same[res.resolved.long()] = True
    assert bool(same.all()), "standalone search != product"
    d = debug_lib()
    import ctypes as C
    info = (C.c_int32 * 3)()
    blocks = (C.c_int64 * 3)()
    d.fwav_debug_topk_plan_info(m, nd, info, blocks)
    geo, mode, P = info[0], info[1], info[2]
    F, R, items = blocks[0], blocks[1], blocks[2]
    qb = int(d.fwav_debug_topk_qb(geo))
    print(f"{a.config}: {m} queries, geometry {geo}, mode {mode}, F {F}, R {R}, P {P}, items {items}, QB {qb}")
    keys = wsk[: items * qb * 256 * 8].view(torch.int64).view(items, qb, 256)
    # the floor's later passes and the overflow relaunches reuse the first key regions (base plans over their lists):
    # skip blocks with any piece there
    from fwav._lib import sim_topk_layout
    lay = sim_topk_layout(m, nd)
    cnt_at = lambda off: int(wsk[off:off + 4].view(torch.int32).item())  # noqa: E731
    n_miss, n_miss2, n_ovf = cnt_at(lay["n_miss"]), cnt_at(lay["n_miss2"]), cnt_at(lay["n_ovf1"])
    nb2 = -(-n_miss // 256)
    reused = max(16 * min(nb2, 64) + max(0, nb2 - 64), -(-n_ovf // 256) + 1)
    print(f"floor misses {n_miss} / {n_miss2}, overflows {n_ovf}: key regions [0, {reused}) reused")
    b0 = max(F, reused)  # pm order: item_of(b, 0) = F + (b - F)
    bs = np.arange(b0, F + R)
    ns, ms, mbs = [], [], []
    for c0 in range(0, len(bs), 32):
        bb = bs[c0:c0 + 32]
        regs = [keys[torch.as_tensor(F + p * R + (bb - F), device=dev)] for p in range(P)]  # (nb, qb, 256) each
        hdr = np.stack([r[:, :, 255].cpu().numpy() for r in regs], -1)  # (nb, qb, P)
        cnt = (hdr & 0xFFFFFFFF).astype(np.int64)
        seed = (hdr >> 32) & 0xFFFFFFFF
        ent = np.stack([r[:, :, :255].cpu().numpy() for r in regs], 2)  # (nb, qb, P, 255)
        valid = np.arange(255)[None, None, None, :] < cnt[..., None]
        hi = ((ent >> 32) & 0xFFFFFFFF).astype(np.int64)
        tp = kth_12(hi, valid)  # (nb, qb, P)
        lkp = np.where(tp > 0, f2key(key2f(tp) - 2 * DELTA).astype(np.int64), 0)
        lk = lkp.max(-1)
        ok = (seed == 0).all(-1)
        uni = valid & (hi > lk[..., None, None])
        mm = uni.reshape(*uni.shape[:2], -1).sum(-1)
        t = kth_12(hi.reshape(*hi.shape[:2], -1), uni.reshape(*uni.shape[:2], -1))
        L = np.maximum(lk, np.where(t > 0, f2key(key2f(t) - 2 * DELTA).astype(np.int64), 0))
        mb = (uni & (hi > L[..., None, None])).reshape(*uni.shape[:2], -1).sum(-1)
        ns.append(cnt.sum(-1)[ok])
        ms.append(mm[ok])
        mbs.append(mb[ok])
    for name, v in (("n (loaded)", np.concatenate(ns)), ("m (> Lk)", np.concatenate(ms)),
                    ("mb (band)", np.concatenate(mbs))):
        q = np.percentile(v, [1, 10, 50, 90, 99, 100])
        print(f"{name:11s} queries {len(v)}: mean {v.mean():.1f}  p1/10/50/90/99/max {np.round(q, 1).tolist()}  "
              f"<=64 {np.mean(v <= 64):.3f} <=128 {np.mean(v <= 128):.3f} <=192 {np.mean(v <= 192):.3f} "
              f"<=256 {np.mean(v <= 256):.3f}")


if __name__ == "__main__":
    main()
