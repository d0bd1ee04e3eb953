"""Rising band limit: K-th tracking by L count levels of width `step` above the limit (counts exact since the last compaction, leapfrogged on each raise), on the real cfg2 table (tools/diag/cent_emb_cfg2.py -> /tmp/cfg2_emb.npy).  usage: python tools/diag/rise_levels_sim.py [n_queries]"""
import sys
import numpy as np
E = np.load('/tmp/cfg2_emb.npy'); nd = len(E); K, C, D = 64, 256, 2e-3
def run(q, L, step, trig=C-32, gran=256):
    s_all = E @ E[q]
    w = s_all[max(0, q - 64):q + 64]
    thf = np.sort(w)[-K] - 2 * D
    buf = []; app = comp = 0; raises = 0
    lv = [thf + 2*D + (j+1)*step for j in range(L)]; cnt = [0]*L
    for a in range(0, nd, gran):
        s = s_all[a:a + gran]
        new = s[s > thf]
        if len(new) == 0: continue
        app += len(new); buf.extend(new.tolist())
        for j in range(L): cnt[j] += int((new > lv[j]).sum())
        # raise to the highest level with K entries
        top = -1
        for j in range(L):
            if cnt[j] >= K: top = j
        if top >= 0:
            raises += 1
            thf = max(thf, lv[top] - 2*D)
            # leapfrog: levels above top stay (their counts are exact since creation), new ones start at 0
            keep_lv = lv[top+1:]; keep_c = cnt[top+1:]
            while len(keep_lv) < L:
                keep_lv.append((keep_lv[-1] if keep_lv else thf + 2*D) + step); keep_c.append(0)
            lv, cnt = keep_lv, keep_c
        if len(buf) > trig:
            comp += 1
            b = np.array(buf); T = np.sort(b)[-K]
            thf = max(thf, T - 2*D); buf = b[b > thf].tolist()
            lv = [thf + 2*D + (j+1)*step for j in range(L)]
            b = np.array(buf); cnt = [int((b > x).sum()) for x in lv]
    return app, comp, raises
n = int(sys.argv[1]); rng = np.random.default_rng(3); qs = rng.choice(330750, n, replace=False)
for L, step in [(0, 1), (2, 4e-3), (4, 2e-3), (8, 4e-3), (8, 8e-3), (16, 4e-3)]:
    r = np.array([run(int(q), L, step) for q in qs])
    print(f"L={L} step={step:g}: appends {r[:,0].mean():6.1f} compactions {r[:,1].mean():5.2f} raises {r[:,2].mean():5.1f}", flush=True)
