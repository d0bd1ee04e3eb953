"""A/B the similarity search of several libfwav builds in ONE process on the same inputs (interleaved rounds).
usage: python tools/ab_topk.py lib1.so lib2.so ..."""
import os as _os_dbg
_os_dbg.environ.setdefault("FWAV_DEBUG_LIBRARY", "1")  # the search knobs: libfwav_debug.so
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
from fwav._lib import SIGNATURES, size_call  # noqa: E402

libs = []
for path in sys.argv[1:]:
    L = C.CDLL(os.path.abspath(path))
    res, args = SIGNATURES["fwav_sim_topk"]
    # builds before round 3 have no blas_threads / ties arguments (and no fwav_tie_check)
    L.new_abi = hasattr(L, "fwav_tie_check")
    if not L.new_abi:
        args = args[:8] + args[9:10] + args[11:]
    L.fwav_sim_topk.restype, L.fwav_sim_topk.argtypes = res, args
    libs.append((os.path.basename(path), L))
cfg = os.environ.get("AB_CFG", "cfg2")  # cfg3: the speech-like 10 min case (its pruned active list)
sig_h, _, _ = synth.make_config_signal(cfg)
tile = synth.CONFIGS[cfg]["tile"]
sig = torch.from_numpy(sig_h).cuda()
# cfg4: only the geometry is needed from the engine run (the harness builds its own table below; searching all
# 21.6 M ranges would take a minute)
r = engine.compress_device(sig, tile, 64, keep_intermediates=True, shard=(0, 256) if cfg == "cfg4" else None)
torch.cuda.synchronize()
nd, nr = r.n_domains, r.n_ranges
rs, step = engine.geometry(tile)
emb16 = torch.empty(2 * ((nd + 255) // 256) * 256 * 16, dtype=torch.float16, device="cuda")
from fwav._lib import call  # noqa: E402
tab = engine.embed_tables(rs, torch.device("cuda"))
pool = torch.empty(nd * rs, device="cuda")
emb = torch.empty(nd * 16, device="cuda")
wsp = size_call("fwav_pool_workspace_size", sig.numel(), tile, rs, step)
ws = torch.empty(max(wsp, 16), dtype=torch.uint8, device="cuda")
st = torch.cuda.current_stream().cuda_stream
call("fwav_pool_embed", sig.data_ptr(), sig.numel(), tile, rs, step, tab.data_ptr(), pool.data_ptr(), emb.data_ptr(),
     emb16.data_ptr(), ws.data_ptr(), ws.numel(), st)
if cfg in ("cfg2", "cfg4"):  # noise: every range active; cfg4 default = one rank's 1/64 of the ranges
    nq = int(os.environ.get("AB_NQ", nr if cfg == "cfg2" else 337_500))  # active queries (default: all ranges)
    active = torch.arange(nq, dtype=torch.int32, device="cuda")
else:  # the engine's own pruned active list
    nq = int(r.n_active.item())
    active = r.active[:nq].clone() if hasattr(r, "active") else torch.arange(nq, dtype=torch.int32, device="cuda")
n_active = torch.tensor([nq], dtype=torch.int32, device="cuda")
# each build's plan (and so its workspace) depends on its own occupancy: size for the largest
wsn = 0
for _, L in libs:
    L.fwav_sim_topk_workspace_size.restype = C.c_size_t
    L.fwav_sim_topk_workspace_size.argtypes = [C.c_int64, C.c_int64, C.c_int]
    if os.environ.get("AB_PLAN"):
        L.fwav_debug_topk_plan(*[int(x) for x in os.environ["AB_PLAN"].split(",")])
    if os.environ.get("AB_GEO"):  # first-pass geometry override (0 base, 1 wide, 2 centroid, 3 centroid wide)
        L.fwav_debug_topk_geometry(int(os.environ["AB_GEO"]))
    wsn = max(wsn, L.fwav_sim_topk_workspace_size(nq, nd, 64))
wsk = torch.empty(wsn, dtype=torch.uint8, device="cuda")
outs = {}
times = {n: [] for n, _ in libs}
plan = os.environ.get("AB_PLAN")  # "rt,pieces": the work-plan override of every build (fwav_debug_topk_plan)
for rnd in range(int(os.environ.get("AB_ROUNDS", 4))):
    for name, L in libs:
        if plan:
            L.fwav_debug_topk_plan(*[int(x) for x in plan.split(",")])
        cand = torch.empty(nr * 64, dtype=torch.int32, device="cuda")
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        extra = (int(os.environ.get("AB_THREADS", 16)),) if L.new_abi else ()
        tie_arg = (None,) if L.new_abi else ()
        rc = L.fwav_sim_topk(emb.data_ptr(), emb16.data_ptr(), nd, active.data_ptr(), n_active.data_ptr(), nq, 0, 64,
                             *extra, cand.data_ptr(), *tie_arg, wsk.data_ptr(), wsn, st)
        e1.record()
        torch.cuda.synchronize()
        assert rc == 0, name
        if rnd > 0:
            times[name].append(e0.elapsed_time(e1))
        # only the searched rows are written (rows past nq, or the pruned ranges' rows of the engine's active list)
        outs[name] = cand[:nq * 64] if cfg in ("cfg2", "cfg4") else cand.view(-1, 64)[active.long()]
        if rnd == 0 and hasattr(L, "fwav_debug_cent_stats"):
            cs = (C.c_ulonglong * 4)()
            L.fwav_debug_cent_stats(cs)
            print(f"{name:24s} centroid filter: {cs[0]} level-1 tiles, {cs[1]} level-2 (tile, set) pairs "
                  f"({cs[1] / max(cs[0], 1):.3f} per tile)", flush=True)
        if rnd == 0:  # overflowed queries of this build: the i32 count at the end of its own workspace layout
            own = L.fwav_sim_topk_workspace_size(nq, nd, 64)
            o = own - 4 - 4 * max(nq, 1)  # ovf list, count, then u32 seeds[q]
            n_ovf = int(wsk[o:o + 4].view(torch.int32).item())
            print(f"{name:24s} active {nq}  overflowed {n_ovf} ({100.0 * n_ovf / max(nq, 1):.1f}%)", flush=True)
ref = outs[libs[0][0]]
for name, _ in libs:
    same = bool(torch.equal(outs[name], ref))
    print(f"{name:24s} median {np.median(times[name]):7.2f} ms  min {min(times[name]):7.2f}  identical={same}", flush=True)
