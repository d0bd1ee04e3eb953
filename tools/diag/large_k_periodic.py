"""Diagnostic: rows where the K=1000 search's first 64 columns differ from the K=64 f32 search (periodic signal)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "audio-compression_amd"), os.path.join(ROOT, "tests")]
import numpy as np
import torch

from fwav import engine

t = np.arange(24000)
sig = np.round(8000 * np.sin(2 * np.pi * t / 32) + 3000 * np.sin(2 * np.pi * 3 * t / 32)).astype(np.float32)
dev = torch.device("cuda", 0)


def cands(K, search):
    r = engine.compress_device(torch.from_numpy(sig).to(dev), 1024, K, keep_intermediates=True, search=search)
    torch.cuda.synchronize()
    return r.cand.cpu().numpy().reshape(-1, K), r


a, r = cands(64, "f32")
for rep in range(2):
    for K in (65, 200, 1000):
        b, _ = cands(K, "f16")
        bad = np.nonzero(~np.all(b[:, :64] == a, axis=1))[0]
        print(f"rep {rep} K={K}: {len(bad)} rows differ", bad[:10])
        if len(bad):
            emb = r.emb.cpu().numpy().reshape(-1, 16)
            i = bad[0]
            q = emb[i]
            sc = emb.astype(np.float64) @ q.astype(np.float64)
            print(" a:", a[i][:12], "\n b:", b[i][:12])
            print(" a scores", sc[a[i][:12]], "\n b scores", sc[b[i][:12]])
            print(" n pruned/zero:", (a[:, 0] < 0).sum(), np.all(emb[:len(a)] == 0, axis=1).sum())
