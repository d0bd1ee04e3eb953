"""Diagnostic: rows where the fp16 search and the all-f32 search disagree on a golden case (tie counts, exact scores
of the differing candidates, and whether the row was re-ranked by fwav.ties)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "audio-compression_amd"), os.path.join(ROOT, "tests")]
import numpy as np
import torch

from fwav import engine, ties
from golden_util import load
from oracle import fractal_oracle as O

case = sys.argv[1]
g = load(case)
p = g["p"]
dev = torch.device("cuda", 0)
T = ties.blas_threads()
print("blas threads", T)
for K in p["Ks"]:
    if K > 64:
        continue
    for order in ("index", "numpy"):
        out = {}
        for search in ("f16", "f32"):
            r = engine.compress_device(torch.from_numpy(g["signal"]).to(dev), p["tile"], K, energy_thresh=p["thr"],
                                       keep_intermediates=True, search=search, tie_order=order)
            torch.cuda.synchronize()
            out[search] = r
            print(case, K, order, search, "n_ties", r.n_ties, "n_resolved", r.n_resolved)
        a = out["f16"].cand.cpu().numpy().reshape(-1, K)
        b = out["f32"].cand.cpu().numpy().reshape(-1, K)
        emb = out["f32"].emb.cpu().numpy().reshape(-1, 16)
        diff = np.nonzero(~np.all(a == b, axis=1))[0]
        print("  rows differing:", len(diff), diff[:20])
        for i in diff[:4]:
            sc = O.sgemv_scores(emb, emb[i][None, :], O.sgemv_col_kind(np.arange(len(emb)), len(emb), T))[0]
            srt = np.sort(sc)[::-1]
            print("   row", i, "K-th", srt[K - 1], "K+1-th", srt[K])
            print("    f16", a[i].tolist())
            print("    f32", b[i].tolist())
            print("    f16 scores", sc[a[i][a[i] >= 0]].tolist())
            print("    f32 scores", sc[b[i][b[i] >= 0]].tolist())
