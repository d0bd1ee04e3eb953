"""A/B the fp16 search's work plan (fwav_debug_topk_plan) in one process on the cfg2 inputs; outputs must be
identical to the unsplit plan.  usage: python tools/plan_ab.py "0:1,512:2,512:3" [seconds]"""
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
from fwav import _lib  # noqa: E402

if os.environ.get("AB_LIB"):  # another build (tools/ab_build.sh)
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import _ablib
    _ablib.use(os.environ["AB_LIB"])

plans = [tuple(int(x) for x in p.split(":")) for p in sys.argv[1].split(",")]
secs = float(sys.argv[2]) if len(sys.argv) > 2 else 60.0
cfgname = os.environ.get("AB_CFG")  # a BASELINE config (cfg3: speech-like, pruned active list) instead of noise
if cfgname:
    sig = torch.from_numpy(synth.make_config_signal(cfgname, seed=0)[0]).cuda()
    tile = synth.CONFIGS[cfgname]["tile"]
else:
    sig = torch.from_numpy(synth.noise(secs, 44100)).cuda()
    tile = 2048
r = engine.compress_device(sig, tile, 64, keep_intermediates=True)
torch.cuda.synchronize()
nd, nr = r.n_domains, r.n_ranges
emb = r.emb
emb16 = torch.empty(size_call("fwav_emb16_elems", nd), dtype=torch.float16, device="cuda")
st = torch.cuda.current_stream().cuda_stream
call("fwav_emb16_from_emb", emb.data_ptr(), nd, emb16.data_ptr(), st)
if os.environ.get("GEOM"):  # first-pass geometry override: 0 = base, 1 = wide
    call("fwav_debug_topk_geometry", int(os.environ["GEOM"]))
if cfgname:
    nq = int(r.n_active.item())
    active = r.active[:nq].clone()
    nr = max(nr, nq)
else:
    nq = int(os.environ.get("AB_NQ", nr))
    active = torch.arange(nq, dtype=torch.int32, device="cuda")
n_active = torch.tensor([nq], dtype=torch.int32, device="cuda")
ref = None
res = []
for rnd in range(3):
    for rt, P in plans:
        call("fwav_debug_topk_plan", rt, P)
        wsn = size_call("fwav_sim_topk_workspace_size", nq, nd, 64)
        wsk = torch.empty(wsn, dtype=torch.uint8, device="cuda")
        cand = torch.empty(nr * 64, dtype=torch.int32, device="cuda")  # rows are indexed by range (active[i])
        ts = []
        for _ in range(3):
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record()
            call("fwav_sim_topk", emb.data_ptr(), emb16.data_ptr(), nd, active.data_ptr(), n_active.data_ptr(), nq, 0,
                 64, 16, cand.data_ptr(), None, wsk.data_ptr(), wsn, st)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        o = wsn - 4 - 4 * max(nq, 1)  # workspace tail: first pass's overflow list, its count, then u32 seeds[q]
        n_ovf = int(wsk[o:o + 4].view(torch.int32).item())
        rows = cand.view(-1, 64)[active.long()]  # only the searched rows are written
        if ref is None:
            ref = rows.clone()
        same = bool(torch.equal(rows, ref))
        if rnd == 2:
            res.append((rt, P, np.median(ts), min(ts), same, wsn, n_ovf))
        del wsk
call("fwav_debug_topk_plan", -1, 1)
for rt, P, med, mn, same, wsn, n_ovf in res:
    print(f"plan rt={rt:5d} P={P}: median {med:7.2f} ms  min {mn:7.2f}  identical={same}  workspace {wsn / 2**30:.2f} GiB  overflowed {n_ovf}",
          flush=True)
