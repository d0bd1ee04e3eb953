"""The cfg2 search's table pieces per block with the speculative floor on (fwav_debug_topk_plan(all blocks, P)),
interleaved on one box: median HIP-event times per P and whether the candidates agree.
usage: [AB_NQ=n] python tools/plan_floor_ab.py [P,P,...] [reps]"""
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

ps = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "-1,4,5,6,8").split(",")]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 7
sig = torch.from_numpy(synth.noise(60.0, 44100)).cuda()
r = engine.compress_device(sig, 2048, 64, keep_intermediates=True)
torch.cuda.synchronize()
nd, nr = r.n_domains, r.n_ranges
st = torch.cuda.current_stream().cuda_stream
emb16 = torch.empty(2 * ((nd + 255) // 256) * 256 * 16, dtype=torch.float16, device="cuda")
call("fwav_emb16_from_emb", r.emb.data_ptr(), nd, emb16.data_ptr(), st)
nq = int(os.environ.get("AB_NQ", nr))
active = torch.arange(nq, dtype=torch.int32, device="cuda")
n_active = torch.tensor([nq], dtype=torch.int32, device="cuda")
times = {p: [] for p in ps}
ref, same = None, True
for rep in range(reps + 1):
    for p in ps:
        call("fwav_debug_topk_plan", -1 if p < 0 else 1 << 20, -1 if p < 0 else p)  # -1: the default plan
        wsn = size_call("fwav_sim_topk_workspace_size", nq, nd, 64)
        wsk = torch.empty(wsn, dtype=torch.uint8, device="cuda")
        cand = torch.empty(nr * 64, dtype=torch.int32, device="cuda")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        call("fwav_sim_topk", r.emb.data_ptr(), emb16.data_ptr(), nd, active.data_ptr(), n_active.data_ptr(), nq, 0, 64,
             16, cand.data_ptr(), None, wsk.data_ptr(), wsn, st)
        e1.record()
        torch.cuda.synchronize()
        if rep:
            times[p].append(e0.elapsed_time(e1))
        ref = cand[:nq * 64].clone() if ref is None else ref
        same = same and bool(torch.equal(cand[:nq * 64], ref))
call("fwav_debug_topk_plan", -1, 1)
for p in ps:
    print(f"{nq} queries, pieces {'default' if p < 0 else p}: median {np.median(times[p]):.3f} ms", flush=True)
print(f"identical={same}", flush=True)
