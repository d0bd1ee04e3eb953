"""Diagnostic: GPU candidates vs the oracle's on a golden case (rows whose candidate sets differ, with scores)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "audio-compression_amd"), os.path.join(ROOT, "tests")]
import numpy as np
import torch

from fwav import engine
from golden_util import load
from oracle import fractal_oracle as O

case, K = sys.argv[1], int(sys.argv[2])
g = load(case)
p = g["p"]
dev = torch.device("cuda", 0)
for search in ("f16", "f32"):
    r = engine.compress_device(torch.from_numpy(g["signal"]).to(dev), p["tile"], K, energy_thresh=p["thr"],
                               keep_intermediates=True, search=search)
    torch.cuda.synchronize()
    cand = r.cand.cpu().numpy().reshape(-1, K)
    emb = r.emb.cpu().numpy().reshape(-1, 16)
    print(search, "emb equals golden emb:", np.array_equal(emb, g["emb"]), "max diff", np.abs(emb - g["emb"]).max())
    pruned = g[f"cand_{K}"][:, 0] < 0
    oc, okth, ok1 = O.topk_candidates(emb, len(cand), K, pruned)
    diff = np.nonzero(~np.all(cand == oc, axis=1))[0]
    print(search, "rows differing from oracle (same emb):", len(diff), diff[:10])
    for i in diff[:3]:
        sc = O.sgemv_scores(emb, emb[i][None, :])[0]
        a, b = set(cand[i].tolist()), set(oc[i].tolist())
        print(" row", i, "gpu-only", [(d, float(sc[d])) for d in a - b], "oracle-only",
              [(d, float(sc[d])) for d in b - a], "kth", okth[i], "k1", ok1[i])
        print("  gpu order", cand[i][:8], " oracle", oc[i][:8])
