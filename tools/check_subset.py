"""Check (tools only): the fp16 search of the first AB_NQ cfg2 queries against the all-f32 kernel — every index in
range, identical candidate rows.  usage: AB_NQ=41344 python tools/check_subset.py [lib.so]"""
import ctypes as C
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "audio-compression_amd")]
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
for nq in [int(x) for x in os.environ.get("AB_NQ", "41344").split(",")]:
    active = torch.arange(nq, dtype=torch.int32, device="cuda")
    n_active = torch.tensor([nq], dtype=torch.int32, device="cuda")
    wsn = L.fwav_sim_topk_workspace_size(nq, nd, 64)
    wsk = torch.empty(wsn, dtype=torch.uint8, device="cuda")
    out = []
    for e16 in (emb16.data_ptr(), None):
        cand = torch.full((nq * 64,), -7, dtype=torch.int32, device="cuda")
        rc = L.fwav_sim_topk(emb.data_ptr(), e16, nd, active.data_ptr(), n_active.data_ptr(), nq, 0, 64, 16,
                             cand.data_ptr(), None, wsk.data_ptr(), wsn, st)
        torch.cuda.synchronize()
        assert rc == 0
        out.append(cand.view(nq, 64))
    c16, c32 = out
    bad = ((c16 < -1) | (c16 >= nd)).any(1)
    diff = (c16 != c32).any(1)
    print(f"nq={nq}: rows with out-of-range entries {int(bad.sum())}, rows differing from f32 {int(diff.sum())}",
          flush=True)
    if bad.any():
        i = int(bad.nonzero()[0])
        print("first bad row", i, c16[i].tolist(), flush=True)
