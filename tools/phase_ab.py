"""Experiment (tools only): two-phase search.  Phase A searches the queries at even list positions as usual; phase B
searches the odd ones with a seed from their neighbours' results: query q scores the domains d + s (s = -2 .. 2
around q − left) of its left neighbour's top K and the mirrored shifts of its right neighbour's, and the K-th best
of those distinct domains (exact f32, minus 2δ) is a valid band limit.  Times A and B with an -DFWAV_TOPK_EXTSEED
build (the seeds come from torch here; a device kernel would compute them) and checks that A ∪ B equals the
one-phase result.  usage: [AB_NQ=...] python tools/phase_ab.py tools/ab/libfwav_ext.so [shifts]
The AB_NQ=41344 run of round 2 ended in a memory fault: this script sized the key workspace for nq queries but
searched nq/2 (a table-pieces plan, which needs more: 258.4 vs 255.6 MB at cfg2), so the kernel wrote past the end
of its workspace.  fwav_debug_sim_topk now takes the workspace size and rejects a short one; the workspace here is
sized for every query count it searches."""
import os as _os_dbg
_os_dbg.environ.setdefault("FWAV_DEBUG_LIBRARY", "1")  # the search knobs: libfwav_debug.so
import ctypes as C
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "audio-compression_amd")]
import numpy as np
import torch

import __graft_entry__

__graft_entry__.build()
from fwav import engine, synth  # noqa: E402
from fwav._lib import SIGNATURES, call, lib  # noqa: E402
L2 = lib()

L = C.CDLL(os.path.abspath(sys.argv[1]))
for n in ("fwav_debug_sim_topk", "fwav_sim_topk_workspace_size"):
    getattr(L, n).restype, getattr(L, n).argtypes = SIGNATURES[n]
shifts = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [-2, -1, 0, 1, 2]
cfg = os.environ.get("AB_CFG", "cfg2")
sig_h, _, _ = synth.make_config_signal(cfg)
tile = synth.CONFIGS[cfg]["tile"]
sig = torch.from_numpy(sig_h).cuda()
r = engine.compress_device(sig, tile, 64, keep_intermediates=True)
torch.cuda.synchronize()
nd, nr = r.n_domains, r.n_ranges
rs, step = engine.geometry(tile)
emb16 = torch.empty(2 * ((nd + 255) // 256) * 256 * 16, dtype=torch.float16, device="cuda")
tab = engine.embed_tables(rs, torch.device("cuda"))
pool = torch.empty(nd * rs, device="cuda")
emb = torch.empty(nd * 16, device="cuda")
ws = torch.empty(max(int(L2.fwav_pool_workspace_size(sig.numel(), tile, rs, step)), 16), dtype=torch.uint8,
                 device="cuda")
st = torch.cuda.current_stream().cuda_stream
call("fwav_pool_embed", sig.data_ptr(), sig.numel(), tile, rs, step, tab.data_ptr(), pool.data_ptr(), emb.data_ptr(),
     emb16.data_ptr(), ws.data_ptr(), ws.numel(), st)
# cfg2: every range; cfg3: the first n_active ranges (as tools/ab_topk.py)
nq = int(os.environ.get("AB_NQ", nr if cfg == "cfg2" else int(r.n_active.item())))
act_all = torch.arange(nq, dtype=torch.int32, device="cuda")
# the plan (and so the key workspace) depends on the query count: size for every count searched below
wsn = max(L.fwav_sim_topk_workspace_size(n, nd, 64) for n in (nq, nq // 2, nq - nq // 2))
wsk = torch.empty(wsn, dtype=torch.uint8, device="cuda")
E = emb.view(nd, 16)
d16 = 2.0e-3


def search(active, seeds=None, reps=4):
    n_active = torch.tensor([active.numel()], dtype=torch.int32, device="cuda")
    cand = torch.full((nr * 64,), -7, dtype=torch.int32, device="cuda")
    times = []
    for rep in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = L.fwav_debug_sim_topk(emb.data_ptr(), emb16.data_ptr(), nd, active.data_ptr(), n_active.data_ptr(),
                                   active.numel(), 0, 64, cand.data_ptr(), wsk.data_ptr(), wsk.numel(), 0,
                                   seeds.data_ptr() if seeds is not None else None, st)
        e1.record()
        torch.cuda.synchronize()
        assert rc == 0
        if rep:
            times.append(e0.elapsed_time(e1))
    return float(np.median(times)), cand.view(nr, 64)


t_full, ref = search(act_all)
A = act_all[0::2].contiguous()
B = act_all[1::2].contiguous()
t_a, ca = search(A)
# seeds of B from the A results
qb = B.long()
left = act_all[0::2][: B.numel()].long()
right_pos = torch.arange(B.numel(), device="cuda") * 2 + 2
has_r = right_pos < act_all.numel()
right = torch.where(has_r, act_all[right_pos.clamp(max=act_all.numel() - 1)].long(), left)
cl = ca[left]                     # (nB, 64)
cr = ca[right]
ol = (qb - left)[:, None]
orr = (right - qb)[:, None]
cands = [cl + ol + s for s in shifts] + [cr - orr + s for s in shifts]
cnd = torch.cat(cands, 1)
valid = torch.cat([(cl >= 0)] * len(shifts) + [(cr >= 0) & has_r[:, None]] * len(shifts), 1)
valid &= (cnd >= 0) & (cnd < nd)
cnd = torch.where(valid, cnd, torch.full_like(cnd, -1))
srt, _ = cnd.sort(1)
dup = torch.zeros_like(srt, dtype=torch.bool)
dup[:, 1:] = srt[:, 1:] == srt[:, :-1]
ok = (srt >= 0) & ~dup
kth = torch.empty(qb.numel(), dtype=torch.float64, device="cuda")
for a0 in range(0, qb.numel(), 16384):
    a1 = min(a0 + 16384, qb.numel())
    sc = (E[qb[a0:a1]][:, None, :].double() * E[srt[a0:a1].clamp(min=0)].double()).sum(-1)
    sc = torch.where(ok[a0:a1], sc, torch.full_like(sc, -float("inf")))
    kth[a0:a1] = sc.topk(64, dim=1).values[:, -1]
seeds = (kth - 2 * d16).float().contiguous()
t_b, cb = search(B, seeds)
t_b0, cb0 = search(B)
got = ref.clone()
got[A.long()] = ca[A.long()]
got[B.long()] = cb[B.long()]
same = bool(torch.equal(got[act_all.long()], ref[act_all.long()]))
exact_k = (E[qb].double() * E[ref[qb][:, 63].long()].double()).sum(1)
gap = (exact_k - kth)[torch.isfinite(kth)]
print(f"{cfg} nq={nq}: one phase {t_full:.2f} ms | A {t_a:.2f} + B seeded {t_b:.2f} = {t_a + t_b:.2f} ms "
      f"(B unseeded {t_b0:.2f}) | seed gap mean {gap.mean().item():.4f} p90 {gap.quantile(0.9).item():.4f} "
      f"no-seed {int((~torch.isfinite(kth)).sum())} | identical={same}", flush=True)
