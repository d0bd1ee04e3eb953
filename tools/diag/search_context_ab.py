"""Diagnostic: the cfg2 search under the engine's calling context (fresh uninitialised workspace, a tie list, the
thread split) against a reused zeroed workspace, with the floor off and on.  usage: python tools/diag/search_context_ab.py"""
import os, sys
os.environ.setdefault("FWAV_DEBUG_LIBRARY", "1")
sys.path[:0] = ["/root/repo", "/root/repo/audio-compression_amd"]
import numpy as np, torch
import __graft_entry__
__graft_entry__.build()
from fwav import engine, synth
from fwav._lib import call, size_call
sig = torch.from_numpy(synth.noise(60.0, 44100)).cuda()
r = engine.compress_device(sig, 2048, 64, keep_intermediates=True)
torch.cuda.synchronize()
nd, nr = r.n_domains, r.n_ranges
st = torch.cuda.current_stream().cuda_stream
emb16 = torch.empty(2 * ((nd + 255) // 256) * 256 * 16, dtype=torch.float16, device="cuda")
call("fwav_emb16_from_emb", r.emb.data_ptr(), nd, emb16.data_ptr(), st)
for nq in (nr, 165375):
    active = torch.arange(nq, dtype=torch.int32, device="cuda")
    n_active = torch.tensor([nq], dtype=torch.int32, device="cuda")
    wsn = size_call("fwav_sim_topk_workspace_size", nq, nd, 64)
    wz = torch.zeros(wsn, dtype=torch.uint8, device="cuda")
    res = {}
    for rep in range(8):
        for floor in (0, -1):
            for ties_on in (0, 1):
                for fresh in (0, 1):
                    for thr in (16, 1):
                        call("fwav_debug_topk_floor", floor, 0.0)
                        ws = torch.empty(wsn, dtype=torch.uint8, device="cuda") if fresh else wz
                        ties = torch.empty(size_call("fwav_tie_list_size", nq), dtype=torch.int32, device="cuda") if ties_on else None
                        cand = torch.empty(nr * 64, dtype=torch.int32, device="cuda")
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0.record()
                        call("fwav_sim_topk", r.emb.data_ptr(), emb16.data_ptr(), nd, active.data_ptr(), n_active.data_ptr(), nq, 0,
                             64, thr, cand.data_ptr(), None if ties is None else ties.data_ptr(), ws.data_ptr(), wsn, st)
                        e1.record()
                        torch.cuda.synchronize()
                        if rep:
                            res.setdefault((floor, ties_on, fresh, thr), []).append(e0.elapsed_time(e1))
                        del ws
    for k, v in sorted(res.items()):
        print(nq, "floor %d ties %d fresh_ws %d threads %d: %.3f ms" % (*k, np.median(v)), flush=True)
