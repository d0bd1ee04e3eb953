"""Slow-path counters of the fp16 search (fwav_debug_sim_topk STATS build) for several libfwav builds on the same
inputs (pool/embeddings from the current library).  usage: [AB_CFG=cfg3] python tools/ab_stats.py lib1.so lib2.so ...
Counters (per wave): replayed chunks, firing tiles, appends/query, compactions/query, tick shares."""
import os as _os_dbg
_os_dbg.environ.setdefault("FWAV_DEBUG_LIBRARY", "1")  # the search knobs: libfwav_debug.so
import ctypes as C
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "audio-compression_amd")]
import torch

import __graft_entry__

__graft_entry__.build()
from fwav import engine, synth  # noqa: E402
from fwav._lib import SIGNATURES, call, size_call  # noqa: E402

cfg = os.environ.get("AB_CFG", "cfg2")
sig_h, _, _ = synth.make_config_signal(cfg)
tile = synth.CONFIGS[cfg]["tile"]
sig = torch.from_numpy(sig_h).cuda()
r = engine.compress_device(sig, tile, 64, keep_intermediates=True)
torch.cuda.synchronize()
nd, nr = r.n_domains, r.n_ranges
rs, step = engine.geometry(tile)
emb16 = torch.empty(size_call("fwav_emb16_elems", nd), dtype=torch.float16, device="cuda")
tab = engine.embed_tables(rs, torch.device("cuda"))
pool = torch.empty(nd * rs, device="cuda")
emb = torch.empty(nd * 16, device="cuda")
wsp = size_call("fwav_pool_workspace_size", sig.numel(), tile, rs, step)
ws = torch.empty(max(wsp, 16), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream().cuda_stream
call("fwav_pool_embed", sig.data_ptr(), sig.numel(), tile, rs, step, tab.data_ptr(), pool.data_ptr(), emb.data_ptr(),
     emb16.data_ptr(), ws.data_ptr(), ws.numel(), st)
nq = int(r.n_active.item())
active = r.active[:nq].clone()
n_active = torch.tensor([nq], dtype=torch.int32, device="cuda")
for path in sys.argv[1:]:
    L = C.CDLL(os.path.abspath(path))
    res, args = SIGNATURES["fwav_debug_sim_topk"]
    L.fwav_debug_sim_topk.restype, L.fwav_debug_sim_topk.argtypes = res, args
    L.fwav_sim_topk_workspace_size.restype = C.c_size_t
    L.fwav_sim_topk_workspace_size.argtypes = [C.c_int64, C.c_int64, C.c_int]
    wsn = L.fwav_sim_topk_workspace_size(nq, nd, 64)
    wsk = torch.empty(wsn, dtype=torch.uint8, device="cuda")
    cand = torch.empty(nr * 64, dtype=torch.int32, device="cuda")
    stats = torch.zeros(16, dtype=torch.int64, device="cuda")
    rc = L.fwav_debug_sim_topk(emb.data_ptr(), emb16.data_ptr(), nd, active.data_ptr(), n_active.data_ptr(), nq, 0,
                               64, cand.data_ptr(), wsk.data_ptr(), wsk.numel(), 0, stats.data_ptr(), st)
    torch.cuda.synchronize()
    assert rc == 0
    sv = stats.cpu().tolist()
    waves = (nq + 255) // 256 * 8
    tot = sv[6]
    print(f"{os.path.basename(path)}: per wave replayed chunks {sv[0] / waves:.1f}, firing tiles {sv[1] / waves:.1f}; "
          f"appends/query {sv[2] / nq:.1f}, compactions/query {sv[3] / nq:.2f}; shares: barrier {sv[7] / tot:.3f}, "
          f"streaming {sv[9] / tot:.3f}, replays {sv[4] / tot:.3f} (compactions {sv[5] / tot:.3f}, appends "
          f"{sv[10] / tot:.3f}), final {sv[8] / tot:.3f}", flush=True)
