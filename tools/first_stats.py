"""Counters of the fp16 search's first pass (STATS build of the kernel: replayed chunks, firing tiles, appends,
compactions, time shares) on cfg2 for the first AB_NQ queries (tools only).
usage: AB_NQ=41344 python tools/first_stats.py   (AB_DBG=262144: the product's geometry instead of the base; 786432: and its floor; AB_RUNS=1: the active
list in runs of 64 in random order, as fwav_prune leaves it)"""
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

if os.environ.get("AB_LIB"):  # counters of another build (tools/ab_build.sh)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import _ablib
    _ablib.use(os.environ["AB_LIB"])

sig_h, _, _ = synth.make_config_signal("cfg2")
sig = torch.from_numpy(sig_h).cuda()
r = engine.compress_device(sig, 2048, 64, keep_intermediates=True)
torch.cuda.synchronize()
nd, nr = r.n_domains, r.n_ranges
st = torch.cuda.current_stream().cuda_stream
emb16 = torch.empty(2 * ((nd + 255) // 256) * 256 * 16, dtype=torch.float16, device="cuda")
tab = engine.embed_tables(8, torch.device("cuda"))
pool = torch.empty(nd * 8, device="cuda")
emb = torch.empty(nd * 16, device="cuda")
ws = torch.empty(max(size_call("fwav_pool_workspace_size", sig.numel(), 2048, 8, 2), 16), dtype=torch.uint8,
                 device="cuda")
call("fwav_pool_embed", sig.data_ptr(), sig.numel(), 2048, 8, 2, tab.data_ptr(), pool.data_ptr(), emb.data_ptr(),
     emb16.data_ptr(), ws.data_ptr(), ws.numel(), st)
if os.environ.get("AB_PLAN"):  # "rt,pieces": the work-plan override (fwav_debug_topk_plan), set before sizing
    call("fwav_debug_topk_plan", *[int(x) for x in os.environ["AB_PLAN"].split(",")])
nq = int(os.environ.get("AB_NQ", nr))
active = torch.arange(nq, dtype=torch.int32, device="cuda")
if os.environ.get("AB_RUNS") == "1":  # fwav_prune's order: runs of 64 consecutive ranges in a random run order
    _g = torch.Generator().manual_seed(0)
    active = torch.cat([torch.arange(r * 64, min(nq, r * 64 + 64), dtype=torch.int32)
                        for r in torch.randperm((nq + 63) // 64, generator=_g).tolist()]).cuda()
n_active = torch.tensor([nq], dtype=torch.int32, device="cuda")
wsn = size_call("fwav_sim_topk_workspace_size", nq, nd, 64)
wsk = torch.empty(wsn, dtype=torch.uint8, device="cuda")
cand = torch.empty(nq * 64, dtype=torch.int32, device="cuda")
for rep in range(2):
    stats = torch.zeros(16, dtype=torch.int64, device="cuda")
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    call("fwav_debug_sim_topk", emb.data_ptr(), emb16.data_ptr(), nd, active.data_ptr(), n_active.data_ptr(), nq, 0,
         64, cand.data_ptr(), wsk.data_ptr(), wsk.numel(), int(os.environ.get("AB_DBG", "0")), stats.data_ptr(), st)
    e1.record()
    torch.cuda.synchronize()
    sv = stats.cpu().tolist()
    qsets = max((nq + 31) // 32, 1)
    tot = max(sv[6], 1)
    print(f"rep {rep}: {e0.elapsed_time(e1):.2f} ms (STATS build); per query set of 32: replayed chunks "
          f"{sv[0] / qsets:.0f}, firing tiles {sv[1] / qsets:.0f}; per query: appends {sv[2] / nq:.1f}, compactions "
          f"{sv[3] / nq:.2f}; shares: barrier {sv[7] / tot:.3f} streaming {sv[9] / tot:.3f} replays {sv[4] / tot:.3f} "
          f"(appends {sv[10] / tot:.3f}, fragment waits {sv[11] / tot:.3f}) final {sv[8] / tot:.3f}; own chunk DMA "
          f"wait {sv[12] / tot:.3f}, compactions {sv[5] / tot:.3f}; centroid: level 1 {sv[13] / tot:.3f}, level-2 pairs "
          f"per query set {sv[14] / qsets:.0f}; busiest wave / mean wave (outside the barrier) "
          f"{sv[15] * int(os.environ.get('AB_W', 8)) / max(sv[6] - sv[7], 1):.3f}", flush=True)
