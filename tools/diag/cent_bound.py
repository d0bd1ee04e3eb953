"""Centroid pre-filter study (round 4): fire rates of group-centroid bounds on the real cfg2 embedding table
(made by tools/diag/cent_emb_cfg2.py into /tmp/cfg2_emb.npy with the oracle).  Output: profiles/r04/cent_sim.log."""
import numpy as np, time
E = np.load('/tmp/cfg2_emb.npy'); nd = len(E); nq = 330750
K = 64; rng = np.random.default_rng(0)
Q = E[:nq]
def kth(qidx):
    S = E @ Q[qidx].T  # nd x g
    return -np.partition(-S, K-1, axis=0)[K-1], S
def eval_groups(groups, label, tile=32):
    fr = []; frq = []
    for g in groups:
        th, S = kth(g)
        c = Q[g].mean(0)
        rt = np.sqrt(((Q[g][:, :8]-c[:8])**2).sum(1)).max(); rr = np.sqrt(((Q[g][:, 8:]-c[8:])**2).sum(1)).max()
        b = E @ c + rt + rr
        thmin = th.min() - 2e-3
        bt = b[: nd//tile*tile].reshape(-1, tile).max(1)
        fr.append((bt > thmin).mean())
        # per query exact tile fire rate (current scheme, final limits)
        st = S[: nd//tile*tile].reshape(-1, tile, len(g)).max(1)
        frq.append((st > th - 2e-3).mean())
        rad = (rt, rr)
    print(f"{label}: group tile fire {np.mean(fr):.4f} (per-query exact tile fire {np.mean(frq):.5f}) last radii {rad[0]:.3f},{rad[1]:.3f}", flush=True)
starts = rng.integers(0, nq-32, 20)
eval_groups([np.arange(s, s+32) for s in starts], "consecutive32")
eval_groups([np.arange(s, s+8) for s in starts], "consecutive8")
eval_groups([np.arange(s, s+4) for s in starts], "consecutive4")
# clustering: k-means on a random-projection sort
t=time.time()
nc = nq//32
C = Q[rng.choice(nq, nc, replace=False)].copy()
for it in range(6):
    # assign (chunks to bound memory)
    a = np.empty(nq, np.int64)
    cn = (C*C).sum(1)
    for i in range(0, nq, 20000):
        a[i:i+20000] = np.argmax(Q[i:i+20000] @ C.T - 0.5*cn, axis=1)
    cnt = np.bincount(a, minlength=nc)
    sums = np.zeros_like(C, dtype=np.float64); np.add.at(sums, a, Q)
    nz = cnt > 0
    C[nz] = (sums[nz]/cnt[nz,None]).astype(np.float32)
    print('kmeans it', it, 'sizes mean', cnt.mean(), 'max', cnt.max(), 'empty', (~nz).sum(), time.time()-t, flush=True)
grp = [np.nonzero(a == j)[0] for j in rng.choice(np.nonzero(cnt >= 16)[0], 20, replace=False)]
print('sizes', [len(g) for g in grp])
eval_groups(grp, "kmeans")
