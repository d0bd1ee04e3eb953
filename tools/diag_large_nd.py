"""Diagnose the similarity search at a large domain count (cfg4-sized table): emb16 layout vs emb, and f16 / f32
kernel candidates vs a torch top-K, for a few queries of a shard."""
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "audio-compression_amd")]
import numpy as np
import torch

import __graft_entry__

__graft_entry__.build()
from fwav import engine, synth  # noqa: E402
from fwav._lib import call  # noqa: E402

secs = float(sys.argv[1]) if len(sys.argv) > 1 else 3600.0
sig = synth.noise(secs, 48000, seed=0)
n = sig.size
rs, tile, K = 8, 2048, 64
nr = -(-n // rs)
lo = nr // 2
m = 256
res = engine.compress_device(torch.from_numpy(sig).cuda(), tile, K, shard=(lo, lo + m), keep_intermediates=True)
torch.cuda.synchronize()
nd = res.n_domains
print("nd", nd, "nr", nr, flush=True)
emb = res.emb.view(-1, 16)
# rebuild emb16 through the public entry point to inspect it
emb16 = torch.empty(2 * ((nd + 255) // 256) * 256 * 16, dtype=torch.float16, device="cuda")
tab = engine.embed_tables(rs, torch.device("cuda"))
from fwav._lib import size_call  # noqa: E402
wsn = size_call("fwav_pool_workspace_size", n, tile, rs, 2)
ws = torch.empty(max(wsn, 16), dtype=torch.uint8, device="cuda")
pool = torch.empty(nd * rs, device="cuda")
emb2 = torch.empty(nd * 16, device="cuda")
sg = torch.from_numpy(sig).cuda()
call("fwav_pool_embed", sg.data_ptr(), n, tile, rs, 2, tab.data_ptr(), pool.data_ptr(), emb2.data_ptr(),
     emb16.data_ptr(), ws.data_ptr(), wsn, torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
e16 = emb16.view(-1, 2, 256, 8).permute(0, 2, 1, 3).reshape(-1, 16)[:nd]
bad = (e16.float() != emb.half().float()).any(dim=1)
print("emb16 rows differing from fp16(emb):", int(bad.sum().item()),
      "first", int(torch.nonzero(bad)[0].item()) if bad.any() else None, flush=True)
cand16 = res.cand.view(m, K).cpu().numpy()
act = torch.arange(m, dtype=torch.int32, device="cuda")
na = torch.tensor([m], dtype=torch.int32, device="cuda")
c32 = torch.full((m * K,), -7, dtype=torch.int32, device="cuda")
call("fwav_sim_topk", emb.data_ptr(), None, nd, act.data_ptr(), na.data_ptr(), m, lo, K, 16, c32.data_ptr(), None, None, 0,
     torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
c32 = c32.view(m, K).cpu().numpy()
print("f16 == f32 rows:", int((cand16 == c32).all(axis=1).sum()), "of", m, flush=True)
for j in (0, 1, 100, 255):
    s = emb @ emb[lo + j]
    top = torch.topk(s, K)
    kth = top.values[-1].item()
    s16 = s[torch.from_numpy(cand16[j].astype(np.int64)).cuda()].min().item()
    s32 = s[torch.from_numpy(c32[j].astype(np.int64)).cuda()].min().item()
    print(f"q{j}: torch kth {kth:.5f}  f16 min {s16:.5f}  f32 min {s32:.5f}  "
          f"f16 max idx {cand16[j].max()}  f32 max idx {c32[j].max()}  torch max idx {top.indices.max().item()}",
          flush=True)


def exact_scores(e, q, idx=None, chunk=1 << 22):
    """f64 elementwise scores (no BLAS)."""
    q = q.double()
    if idx is not None:
        return (e[idx].double() * q).sum(-1)
    out = torch.empty(e.shape[0], dtype=torch.float64, device=e.device)
    for a in range(0, e.shape[0], chunk):
        out[a:a + chunk] = (e[a:a + chunk].double() * q).sum(-1)
    return out


for j in (0, 255):
    q = emb[lo + j]
    s64 = exact_scores(emb, q)
    top = torch.topk(s64, K)
    ours = exact_scores(emb, q, torch.from_numpy(cand16[j].astype(np.int64)).cuda())
    sg = emb @ q
    print(f"q{j} exact: kth {top.values[-1].item():.5f} (max idx {top.indices.max().item()}), ours min "
          f"{ours.min().item():.5f}; torch gemv vs exact max |diff| {(sg.double() - s64).abs().max().item():.3g} "
          f"at {int((sg.double() - s64).abs().argmax().item())}", flush=True)
