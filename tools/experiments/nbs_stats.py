"""Counters of neighbour seeding (tools only, an -DFWAV_TOPK_NBSTATS build): odd-position queries tried, those with a
finished neighbour row, those seeded, and the mean seed; next to the exact K-th scores.  usage:
python tools/nbs_stats.py tools/ab/libfwav_nbstats.so"""
import ctypes as C
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "audio-compression_amd")]
import torch

import __graft_entry__

__graft_entry__.build()
from fwav import _lib, engine, synth  # noqa: E402

_lib.LIB_PATH = os.path.abspath(sys.argv[1])
_lib._lib = None
L = _lib.lib()
L.fwav_debug_nbs_stats.restype = C.c_int
L.fwav_debug_nbs_stats.argtypes = [C.c_void_p, C.c_int]
sig = torch.from_numpy(synth.make_config_signal("cfg2")[0]).cuda()
h = (C.c_ulonglong * 4)()
for rep in range(3):
    L.fwav_debug_nbs_stats(h, 1)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    r = engine.compress_device(sig, 2048, 64, keep_intermediates=True)
    e1.record()
    torch.cuda.synchronize()
    L.fwav_debug_nbs_stats(h, 0)
    print(f"rep {rep}: step {e0.elapsed_time(e1):.2f} ms; odd queries tried {h[0]}, with a neighbour row {h[1]}, "
          f"seeded {h[2]}, mean seed {h[3] / max(h[2], 1) / 1e6:.4f}", flush=True)
E = r.emb.view(-1, 16)
c = r.cand.view(-1, 64)
kth = (E[:c.shape[0]].double() * E[c[:, 63].long()].double()).sum(1)
print(f"exact K-th: mean {kth.mean().item():.4f} (seed − 2δ expected ≈ {kth.mean().item() - 0.004:.4f})")
