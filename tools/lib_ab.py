"""Same-process A/B of two builds of the search (e.g. the debug library against a tools/ab_build.sh variant): the
cfg2 search (fwav_sim_topk, default knobs) alternated between the libraries, median HIP-event times per library and
whether the candidates agree.  usage: [AB_NQ=n] python tools/lib_ab.py LIB_A LIB_B [reps]"""
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
from fwav._lib import SIGNATURES  # noqa: E402

libs = []
for path in sys.argv[1:3]:
    L = C.CDLL(os.path.abspath(path))
    for n in ("fwav_sim_topk", "fwav_sim_topk_workspace_size", "fwav_emb16_from_emb", "fwav_last_error"):
        getattr(L, n).restype, getattr(L, n).argtypes = SIGNATURES[n]
    libs.append(L)
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 9
sig = torch.from_numpy(synth.noise(60.0, 44100)).cuda()
r = engine.compress_device(sig, 2048, 64, keep_intermediates=True)
torch.cuda.synchronize()
nd, nr = r.n_domains, r.n_ranges
st = torch.cuda.current_stream().cuda_stream
emb16 = torch.empty(2 * ((nd + 255) // 256) * 256 * 16, dtype=torch.float16, device="cuda")
assert libs[0].fwav_emb16_from_emb(r.emb.data_ptr(), nd, emb16.data_ptr(), st) == 0
nq = int(os.environ.get("AB_NQ", nr))
active = torch.arange(nq, dtype=torch.int32, device="cuda")
n_active = torch.tensor([nq], dtype=torch.int32, device="cuda")
wsn = max(L.fwav_sim_topk_workspace_size(nq, nd, 64) for L in libs)
wsk = torch.empty(wsn, dtype=torch.uint8, device="cuda")
times = [[], []]
cands = [None, None]
for rep in range(reps + 1):
    for i, L in enumerate(libs):
        cand = torch.empty(nr * 64, dtype=torch.int32, device="cuda")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = L.fwav_sim_topk(r.emb.data_ptr(), emb16.data_ptr(), nd, active.data_ptr(), n_active.data_ptr(), nq, 0, 64,
                             16, cand.data_ptr(), None, wsk.data_ptr(), wsn, st)
        e1.record()
        torch.cuda.synchronize()
        assert rc == 0, L.fwav_last_error()
        if rep:
            times[i].append(e0.elapsed_time(e1))
        cands[i] = cand[:nq * 64]
for i in range(2):
    print(f"{sys.argv[1 + i]}: {nq} queries, median {np.median(times[i]):.3f} ms (min {min(times[i]):.3f})", flush=True)
print(f"identical={bool(torch.equal(cands[0], cands[1]))}", flush=True)
