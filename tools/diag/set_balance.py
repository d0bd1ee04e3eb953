"""How much of the centroid kernel's group-barrier wait a re-pairing of query sets to waves could remove: runs the
cfg2 first pass of a -DFWAV_TOPK_SETSTATS debug build once and reads, per item, each wave's total and barrier-wait
ticks and each query set's level-2 + append ticks.  Reports per item the busiest / mean wave busy time as run, and
as it would be with the 16 sets re-paired heavy-with-light (a wave keeps its own uniform part: level 1 etc.).
usage: AB_LIB=tools/ab/libfwav_setstats.so python tools/diag/set_balance.py"""
import ctypes as C
import os
import sys

os.environ.setdefault("FWAV_DEBUG_LIBRARY", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "audio-compression_amd"), os.path.join(ROOT, "tools")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import __graft_entry__  # noqa: E402

__graft_entry__.build()
from fwav import engine, synth  # noqa: E402
from fwav._lib import call, size_call  # noqa: E402
import _ablib  # noqa: E402

lib = C.CDLL(os.path.abspath(os.environ["AB_LIB"]))
lib.fwav_debug_set_stats.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
lib.fwav_debug_set_stats.restype = C.c_int
_ablib.use(os.environ["AB_LIB"])
sig = torch.from_numpy(synth.noise(60.0, 44100)).cuda()
r = engine.compress_device(sig, 2048, 64, keep_intermediates=True)
torch.cuda.synchronize()
nd, nr = r.n_domains, r.n_ranges
nq = int(os.environ.get("AB_NQ", nr))
active = torch.arange(nq, dtype=torch.int32, device="cuda")
n_active = torch.tensor([nq], dtype=torch.int32, device="cuda")
cand = torch.empty(nr * 64, dtype=torch.int32, device="cuda")
ws = torch.empty(size_call("fwav_sim_topk_workspace_size", nq, nd, 64), dtype=torch.uint8, device="cuda")
emb16 = torch.empty(2 * ((nd + 255) // 256) * 256 * 16, dtype=torch.float16, device="cuda")
call("fwav_emb16_from_emb", r.emb.data_ptr(), nd, emb16.data_ptr(), torch.cuda.current_stream().cuda_stream)
for _ in range(2):
    call("fwav_sim_topk", r.emb.data_ptr(), emb16.data_ptr(), nd, active.data_ptr(), n_active.data_ptr(), nq, 0, 64, 16,
         cand.data_ptr(), None, ws.data_ptr(), ws.numel(), torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
sets = np.zeros(1 << 16, np.uint64)
waits = np.zeros(1 << 16, np.uint64)
tot = np.zeros(1 << 16, np.uint64)
lib.fwav_debug_set_stats(sets.ctypes.data, waits.ctypes.data, tot.ctypes.data)
W, NG = 8, 16
items = int(np.count_nonzero(tot)) // W
T = tot[:items * W].reshape(items, W).astype(np.float64)
Wt = waits[:items * W].reshape(items, W).astype(np.float64)
S = sets[:items * NG].reshape(items, NG).astype(np.float64)
busy = T - Wt
own = S.reshape(items, W, 2).sum(-1)
uni = busy - own
now = (busy.max(1) / busy.mean(1))
rep = []
for i in range(items):
    o = np.sort(S[i])
    pairs = o[:W] + o[::-1][:W]  # heavy with light
    b2 = uni[i].mean() + pairs
    rep.append(b2.max() / b2.mean())
rep = np.array(rep)
print(f"{items} items; wave time: barrier wait {Wt.sum() / T.sum():.1%}, set work (level 2 + appends) "
      f"{S.sum() / T.sum():.1%} of wave time; uniform part (level 1, shared limits, final) {uni.sum() / T.sum():.1%}")
print(f"busiest / mean wave busy time per item: as run {now.mean():.3f} (median {np.median(now):.3f}); "
      f"sets re-paired heavy-with-light {rep.mean():.3f}")
cv = S.std(1) / S.mean(1)
print(f"per-item coefficient of variation of set work: mean {cv.mean():.3f}")
