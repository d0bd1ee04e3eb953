"""Run the cfg2 similarity search once (after one warm-up) with a given dbg value — a target for rocprofv3 --pmc.
usage: [AB_NQ=n] [AB_GEO=g] [AB_LIB=lib] python tools/topk_once.py [dbg]"""
import os as _os_dbg
_os_dbg.environ.setdefault("FWAV_DEBUG_LIBRARY", "1")  # the search knobs: libfwav_debug.so
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "audio-compression_amd")]
import torch

import __graft_entry__

__graft_entry__.build()
from fwav import engine, synth  # noqa: E402
from fwav import _lib  # noqa: E402
from fwav._lib import call, size_call  # noqa: E402

if os.environ.get("AB_LIB"):  # another build (tools/ab_build.sh), e.g. for PMC passes of a variant
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import _ablib
    _ablib.use(os.environ["AB_LIB"])

dbg = int(sys.argv[1]) if len(sys.argv) > 1 else 0
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
nq = int(os.environ.get("AB_NQ", nr))  # active queries (the first nq ranges; default all)
if os.environ.get("AB_GEO"):  # first-pass geometry override (0 base, 1 wide, 2 centroid, 3 centroid wide)
    call("fwav_debug_topk_geometry", int(os.environ["AB_GEO"]))
active = torch.arange(nq, dtype=torch.int32, device="cuda")
n_active = torch.tensor([nq], dtype=torch.int32, device="cuda")
cand = torch.empty(nr * 64, dtype=torch.int32, device="cuda")
wsk = torch.empty(size_call("fwav_sim_topk_workspace_size", nq, nd, 64), dtype=torch.uint8, device="cuda")
for _ in range(2):
    call("fwav_debug_sim_topk", emb.data_ptr(), emb16.data_ptr(), nd, active.data_ptr(), n_active.data_ptr(), nq, 0,
         64, cand.data_ptr(), wsk.data_ptr(), wsk.numel(), dbg, None, st)
torch.cuda.synchronize()
print("done", dbg)
