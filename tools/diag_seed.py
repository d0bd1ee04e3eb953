"""Diagnose the seeded fp16 search against the f32 kernel on a golden case (tools only).
usage: python tools/diag_seed.py [case] [K]"""
import os as _os_dbg
_os_dbg.environ.setdefault("FWAV_DEBUG_LIBRARY", "1")  # the search knobs: libfwav_debug.so
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "audio-compression_amd"),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests")]
import numpy as np
import torch

import __graft_entry__

__graft_entry__.build()
from fwav import engine  # noqa: E402
from fwav._lib import call, size_call  # noqa: E402
from golden_util import load  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "sweep"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 64
g = load(case)
p = g["p"]
sig = torch.from_numpy(g["signal"]).cuda()
r = engine.compress_device(sig, p["tile"], K, energy_thresh=p["thr"], keep_intermediates=True, search="f32")
torch.cuda.synchronize()
ref = r.cand.cpu().numpy().reshape(-1, K)
nd, nr = r.n_domains, r.n_ranges
emb = r.emb
rs = r.pool.numel() // nd
step = r.domain_step if hasattr(r, "domain_step") else None
from oracle import fractal_oracle as O  # noqa: E402  (tools: geometry only)
rs2, step = O.geometry(p["tile"])[:2]
assert rs2 == rs
emb16 = torch.empty(2 * ((nd + 255) // 256) * 256 * 16, dtype=torch.float16, device="cuda")
tab = engine.embed_tables(rs, torch.device("cuda"))
pool = torch.empty(nd * rs, device="cuda")
emb2 = torch.empty(nd * 16, device="cuda")
ws = torch.empty(size_call("fwav_pool_workspace_size", sig.numel(), p["tile"], rs, step), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream().cuda_stream
call("fwav_pool_embed", sig.data_ptr(), sig.numel(), p["tile"], rs, step, tab.data_ptr(), pool.data_ptr(),
     emb2.data_ptr(), emb16.data_ptr(), ws.data_ptr(), ws.numel(), st)
print("nd", nd, "nr", nr, "rs", rs)
active = torch.arange(nr, dtype=torch.int32, device="cuda")
n_active = torch.tensor([nr], dtype=torch.int32, device="cuda")
E = emb.cpu().numpy().reshape(-1, 16).astype(np.float64)
for plan in [(0, 1), (-1, 1)]:
    call("fwav_debug_topk_plan", *plan)
    wsn = size_call("fwav_sim_topk_workspace_size", nr, nd, K)
    wsk = torch.empty(wsn, dtype=torch.uint8, device="cuda")
    for dbg in (-1, 0, 8192):
        cand = torch.full((nr * K,), -7, dtype=torch.int32, device="cuda")
        if dbg < 0:  # production kernel
            call("fwav_sim_topk", emb.data_ptr(), emb16.data_ptr(), nd, active.data_ptr(), n_active.data_ptr(), nr, 0,
                 K, 16, cand.data_ptr(), None, wsk.data_ptr(), wsn, st)
        else:
            call("fwav_debug_sim_topk", emb.data_ptr(), emb16.data_ptr(), nd, active.data_ptr(), n_active.data_ptr(),
                 nr, 0, K, cand.data_ptr(), wsk.data_ptr(), wsk.numel(), dbg | 16384, None, st)
        torch.cuda.synchronize()
        c = cand.cpu().numpy().reshape(-1, K)
        bad = np.nonzero(~np.all(c == ref, axis=1))[0]
        wb = wsk.cpu().numpy()
        o = wsn - 4 - 4 * nr  # ovf list, its count, then u32 seeds[q]
        n_ovf = int(wb[o:o + 4].view(np.int32)[0])
        ovf = wb[o - 4 * nr:o].view(np.int32)[:n_ovf]
        print(f"   n_ovf {n_ovf}: bad rows in ovf list: {np.isin(bad, ovf).sum()} of {len(bad)}; ovf[:12] {np.sort(ovf)[:12]}")
        print(f"plan {plan} dbg {dbg}: {len(bad)} rows differ from f32", bad[:10])
        for q in bad[:3]:
            s = E @ E[q]
            print("   q", q, "missing", sorted(set(ref[q]) - set(c[q]))[:8], "extra", sorted(set(c[q]) - set(ref[q]))[:8],
                  "kth", np.sort(s)[::-1][K - 1], "n(-1)", int((c[q] < 0).sum()))
call("fwav_debug_topk_plan", 0, 1)
wsn = size_call("fwav_sim_topk_workspace_size", nr, nd, K)
wsk = torch.empty(wsn, dtype=torch.uint8, device="cuda")
stats = torch.zeros(16 + nr + 512, dtype=torch.int64, device="cuda")
cand = torch.full((nr * K,), -7, dtype=torch.int32, device="cuda")
call("fwav_debug_sim_topk", emb.data_ptr(), emb16.data_ptr(), nd, active.data_ptr(), n_active.data_ptr(), nr, 0, K,
     cand.data_ptr(), wsk.data_ptr(), wsk.numel(), 32768, stats.data_ptr(), st)
torch.cuda.synchronize()
seeds = stats[16:16 + nr].cpu().numpy().astype(np.uint32).view(np.float32)
E16 = emb16.cpu().numpy().reshape(-1, 2, 256, 8).transpose(0, 2, 1, 3).reshape(-1, 16)[:nd].astype(np.float64)
for q in (67, 68, 69, 180, 1000):
    s = E @ E[q]
    s16 = E16 @ E16[q]
    w = np.sort(s16[max(0, q - 64):q + 64])[::-1]
    kth = np.sort(s)[::-1][K - 1]
    print(f"q {q}: seed {seeds[q]:.6f}  window K-th s16 {w[K - 1]:.6f} -2d {w[K - 1] - 5e-3:.6f}  true kth {kth:.6f}  "
          f"min s16 of true top-K {s16[np.argsort(-s, kind='stable')[:K]].min():.6f}")
call("fwav_debug_topk_plan", -1, 1)
