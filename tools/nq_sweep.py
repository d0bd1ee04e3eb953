"""Timing (tools only): the fp16 search of the first nq cfg2 queries for a list of nq (round structure of the
work plan: 256 queries per block, 2 blocks per CU).  usage: AB_NQ=131072,262144,330750 python tools/nq_sweep.py [lib]"""
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
from fwav._lib import SIGNATURES, call, lib, size_call  # noqa: E402

L = C.CDLL(os.path.abspath(sys.argv[1])) if len(sys.argv) > 1 else lib()
for n in ("fwav_sim_topk", "fwav_sim_topk_workspace_size"):
    getattr(L, n).restype, getattr(L, n).argtypes = SIGNATURES[n]
sig = torch.from_numpy(synth.make_config_signal("cfg2")[0]).cuda()
r = engine.compress_device(sig, 2048, 64, keep_intermediates=True)
torch.cuda.synchronize()
nd, nr = r.n_domains, r.n_ranges
emb16 = torch.empty(2 * ((nd + 255) // 256) * 256 * 16, dtype=torch.float16, device="cuda")
tab = engine.embed_tables(8, torch.device("cuda"))
pool = torch.empty(nd * 8, device="cuda")
emb = torch.empty(nd * 16, device="cuda")
ws = torch.empty(max(size_call("fwav_pool_workspace_size", sig.numel(), 2048, 8, 2), 16), dtype=torch.uint8,
                 device="cuda")
st = torch.cuda.current_stream().cuda_stream
call("fwav_pool_embed", sig.data_ptr(), sig.numel(), 2048, 8, 2, tab.data_ptr(), pool.data_ptr(), emb.data_ptr(),
     emb16.data_ptr(), ws.data_ptr(), ws.numel(), st)
for nq in [int(x) for x in os.environ.get("AB_NQ", "131072,262144,330750").split(",")]:
    active = torch.arange(nq, dtype=torch.int32, device="cuda")
    n_active = torch.tensor([nq], dtype=torch.int32, device="cuda")
    wsn = L.fwav_sim_topk_workspace_size(nq, nd, 64)
    wsk = torch.empty(wsn, dtype=torch.uint8, device="cuda")
    cand = torch.empty(nq * 64, dtype=torch.int32, device="cuda")
    times = []
    for rep in range(5):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = L.fwav_sim_topk(emb.data_ptr(), emb16.data_ptr(), nd, active.data_ptr(), n_active.data_ptr(), nq, 0, 64,
                             16, cand.data_ptr(), None, wsk.data_ptr(), wsn, st)
        e1.record()
        torch.cuda.synchronize()
        assert rc == 0
        if rep:
            times.append(e0.elapsed_time(e1))
    t = float(np.median(times))
    print(f"nq={nq:7d} blocks={(nq + 255) // 256:5d}: {t:7.2f} ms  ({t / nq * 1e6:.1f} ns/query)", flush=True)
