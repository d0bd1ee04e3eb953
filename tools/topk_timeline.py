"""Workgroup timeline of the similarity search (dbg 4096): how busy the GPU's workgroup slots are over time.
usage: [PLAN=rt:P] [AB_NQ=n] python tools/topk_timeline.py [dbg_extra]   (AB_NQ: the first n queries only)   (prints occupancy profile + the tail's share of the kernel)"""
import os as _os_dbg
_os_dbg.environ.setdefault("FWAV_DEBUG_LIBRARY", "1")  # the search knobs: libfwav_debug.so
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "audio-compression_amd")]
import numpy as np
import torch

import __graft_entry__

__graft_entry__.build()
from fwav import engine, synth  # noqa: E402
from fwav._lib import call, size_call  # noqa: E402

extra = int(sys.argv[1]) if len(sys.argv) > 1 else 0
if os.environ.get("PLAN"):  # "rt:P" work-plan override
    call("fwav_debug_topk_plan", *[int(x) for x in os.environ["PLAN"].split(":")])
sig = torch.from_numpy(synth.noise(60.0, 44100)).cuda()
r = engine.compress_device(sig, 2048, 64, keep_intermediates=True)
torch.cuda.synchronize()
nd, nr = r.n_domains, r.n_ranges
emb16 = torch.empty(2 * ((nd + 255) // 256) * 256 * 16, dtype=torch.float16, device="cuda")
tab = engine.embed_tables(8, torch.device("cuda"))
pool = torch.empty(nd * 8, device="cuda")
emb = torch.empty(nd * 16, device="cuda")
ws = torch.empty(16 << 20, dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream().cuda_stream
call("fwav_pool_embed", sig.data_ptr(), sig.numel(), 2048, 8, 2, tab.data_ptr(), pool.data_ptr(), emb.data_ptr(),
     emb16.data_ptr(), ws.data_ptr(), ws.numel(), st)
nr = int(os.environ.get("AB_NQ", nr))
active = torch.arange(nr, dtype=torch.int32, device="cuda")
n_active = torch.tensor([nr], dtype=torch.int32, device="cuda")
cand = torch.empty(nr * 64, dtype=torch.int32, device="cuda")
wsk = torch.empty(size_call("fwav_sim_topk_workspace_size", nr, nd, 64), dtype=torch.uint8, device="cuda")
nblk = 8192
stats = torch.zeros(16 + 2 * nblk, dtype=torch.int64, device="cuda")
for _ in range(2):
    stats.zero_()
    stats[16::2] = 2**62
    call("fwav_debug_sim_topk", emb.data_ptr(), emb16.data_ptr(), nd, active.data_ptr(), n_active.data_ptr(), nr, 0,
         64, cand.data_ptr(), wsk.data_ptr(), wsk.numel(), 4096 | extra, stats.data_ptr(), st)
    torch.cuda.synchronize()
tl = stats[16:].cpu().numpy().reshape(-1, 2)
tl = tl[tl[:, 0] < 2**62].astype(np.float64)
t0 = tl[:, 0].min()
s, e = (tl[:, 0] - t0) / 100.0, (tl[:, 1] - t0) / 100.0  # µs (100 MHz ticks)
T = e.max()
print(f"{len(tl)} workgroups, kernel span {T / 1000:.2f} ms, WG duration median {np.median(e - s) / 1000:.2f} ms "
      f"p10 {np.percentile(e - s, 10) / 1000:.2f} p90 {np.percentile(e - s, 90) / 1000:.2f}")
grid = np.linspace(0, T, 41)
for a, b in zip(grid[:-1], grid[1:]):
    m = (a + b) / 2
    print(f"  t={m / 1000:6.2f} ms  busy WGs {int(((s <= m) & (e > m)).sum()):4d}")
busy = sum(e - s)
print(f"slot-time utilisation vs 512 slots: {busy / (512 * T):.3f}")
ids = np.nonzero(stats[16:].cpu().numpy().reshape(-1, 2)[:, 0] < 2**62)[0]
order = np.argsort(-e)[:12]
print("latest-ending workgroups (block, start ms, end ms, duration ms):")
for i in order:
    print(f"  {ids[i]:5d} {s[i] / 1000:6.2f} {e[i] / 1000:6.2f} {(e[i] - s[i]) / 1000:6.2f}")
order = np.argsort(-(e - s))[:12]
print("longest workgroups:")
for i in order:
    print(f"  {ids[i]:5d} {s[i] / 1000:6.2f} {e[i] / 1000:6.2f} {(e[i] - s[i]) / 1000:6.2f}")
# duration of the workgroups that start with the launch (first round, all in the same phase) vs the later ones
first = s < 50.0
print(f"first-round workgroups {int(first.sum())}: median duration {np.median((e - s)[first]) / 1000:.2f} ms; "
      f"later {int((~first).sum())}: median {np.median((e - s)[~first]) / 1000:.2f} ms")
if os.environ.get("TL_R"):  # piece-major plan with R split blocks from item 0: median duration per table piece
    R = int(os.environ["TL_R"])
    dur = (e - s) / 1000
    for p in range(int(ids.max()) // R + 1):
        sel = (ids // R) == p
        if sel.any():
            print(f"piece {p}: {int(sel.sum())} items, duration median {np.median(dur[sel]):.2f} ms, "
                  f"max {dur[sel].max():.2f}")
