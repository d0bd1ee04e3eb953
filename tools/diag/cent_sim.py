"""Centroid pre-filter study (round 4): fire rates of group-centroid bounds on the real cfg2 embedding table
(made by tools/diag/cent_emb_cfg2.py into /tmp/cfg2_emb.npy with the oracle).  Output: profiles/r04/cent_sim.log."""
import numpy as np, sys
E = np.load('/tmp/cfg2_emb.npy'); nd = len(E); nq = 330750; K = 64
d16 = 2e-3
def sim(q0, g=4, nsets=4, win_chunks=128, warm=32):
    Q = E[q0:q0+32*nsets]                     # nsets sets of 32 consecutive queries
    nqq = len(Q)
    C = Q.reshape(-1, g, 16).mean(1)           # centroids of g consecutive queries
    rt = np.sqrt(((Q.reshape(-1,g,16)[:,:,:8]-C[:,None,:8])**2).sum(2)).max(1)
    rr = np.sqrt(((Q.reshape(-1,g,16)[:,:,8:]-C[:,None,8:])**2).sum(2)).max(1)
    rho = rt + rr
    # seeds: K-th within own window +-64
    th = np.empty(nqq, np.float32)
    for i in range(nqq):
        qi = q0 + i
        w = E[max(0, qi-64):qi+64] @ Q[i]
        th[i] = np.sort(w)[-K] - 2*d16 if len(w) >= K else -np.inf
    top = None
    nch = -(-nd // 256)
    lvl1 = 0; lvl2 = 0; cur = 0; fires_q = 0
    t = 0
    chunk = 0
    while chunk < nch:
        span = warm if chunk < warm else win_chunks  # limits update every span (approx: every group during warm)
        step = 4 if chunk < warm else span
        c1 = min(nch, chunk + step)
        S = E[chunk*256: c1*256] @ Q.T          # domains x queries
        Sc = E[chunk*256: c1*256] @ C.T
        ntile = -(-S.shape[0] // 32)
        pad = ntile*32 - S.shape[0]
        if pad:
            S = np.vstack([S, np.full((pad, nqq), -9, np.float32)]); Sc = np.vstack([Sc, np.full((pad, len(C)), -9, np.float32)])
        tm = S.reshape(ntile, 32, nqq).max(1)      # tile max per query
        tcm = Sc.reshape(ntile, 32, len(C)).max(1)
        T = th.reshape(-1, g).min(1) - rho - 2*d16
        cf = tcm > T[None, :]                      # centroid fires
        sf = cf.reshape(ntile, nsets, -1).any(2)   # set fires
        lvl1 += ntile; lvl2 += sf.sum()
        fires_q += (tm > th[None, :]).sum()
        # update limits: K-th of everything so far (exact; kept K per query)
        blk = S[:S.shape[0]-pad] if pad else S
        allv = blk if top is None else np.vstack([top, blk])
        top = -np.partition(-allv, K-1, axis=0)[:K]
        th = np.maximum(th, top[K-1] - 2*d16)
        chunk = c1
    return lvl1, lvl2, fires_q, rho.mean()
for q0 in [1000, 90000, 200000, 300000]:
    for g in (2, 4, 8):
        nsets = {2:2, 4:4, 8:8}[g]
        l1, l2, f, r = sim(q0, g, nsets)
        cur = l1 * nsets
        new = l1 + l2
        print(f"q0 {q0} g {g}: tiles {l1} level2 set-tiles {l2} ({l2/l1/nsets:.3f} of sets), work new/cur {new/cur:.3f}, rho {r:.3f}", flush=True)
