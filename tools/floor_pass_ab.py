"""The speculative floor's A/B (fwav_debug_topk_floor): the cfg2 search (fwav_sim_topk through libfwav_debug.so) with
the floor off (0) and by default (-1), interleaved, at the full query count and at one rank's share of N = 8
(41,344 queries); reports median HIP-event times, the pilots' floor, the second pass's miss count (read from the
workspace tail) and whether the candidates are identical.
usage: [AB_SIZES=n1,n2] [AB_CONFIGS=mode:value,...] [AB_GEN=speech] python tools/floor_pass_ab.py [reps]"""
import os as _os_dbg
_os_dbg.environ.setdefault("FWAV_DEBUG_LIBRARY", "1")  # the search knobs: libfwav_debug.so
import os
import struct
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "audio-compression_amd")]
import numpy as np
import torch

import __graft_entry__

__graft_entry__.build()
from fwav import engine, synth  # noqa: E402
from fwav._lib import call, size_call  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 7
sig = torch.from_numpy((synth.speech_like if os.environ.get("AB_GEN") == "speech" else synth.noise)(60.0, 44100)).cuda()
r = engine.compress_device(sig, 2048, 64, keep_intermediates=True)
torch.cuda.synchronize()
nd, nr = r.n_domains, r.n_ranges
st = torch.cuda.current_stream().cuda_stream
emb16 = torch.empty(2 * ((nd + 255) // 256) * 256 * 16, dtype=torch.float16, device="cuda")
call("fwav_emb16_from_emb", r.emb.data_ptr(), nd, emb16.data_ptr(), st)
TAIL = 4 * (1024 * 512 * 8 + 512) + 8  # after the second miss list's count: two floor keys, the pilots' scores
CONFIGS = [tuple(map(float, c.split(":"))) for c in os.environ.get("AB_CONFIGS", "0:0,-1:0,2:1,2:3,2:10,2:20").split(",")]  # (mode, value): off, default, ranks
SIZES = [int(x) for x in os.environ.get("AB_SIZES", f"{nr},41344").split(",")]  # query counts (first nq ranges)
for nq in SIZES:
    active = torch.arange(nq, dtype=torch.int32, device="cuda")
    n_active = torch.tensor([nq], dtype=torch.int32, device="cuda")
    wsn = size_call("fwav_sim_topk_workspace_size", nq, nd, 64)
    wsk = torch.zeros(wsn, dtype=torch.uint8, device="cuda")
    times = {c: [] for c in CONFIGS}
    info = {}
    ref = None
    same = True
    for rep in range(reps + 1):
        for c in CONFIGS:
            call("fwav_debug_topk_floor", int(c[0]), c[1])
            cand = torch.empty(nr * 64, dtype=torch.int32, device="cuda")
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            call("fwav_sim_topk", r.emb.data_ptr(), emb16.data_ptr(), nd, active.data_ptr(), n_active.data_ptr(), nq, 0,
                 64, 16, cand.data_ptr(), None, wsk.data_ptr(), wsn, st)
            e1.record()
            torch.cuda.synchronize()
            if rep:
                times[c].append(e0.elapsed_time(e1))
            if ref is None:
                ref = cand[:nq * 64].clone()
            same = same and bool(torch.equal(cand[:nq * 64], ref))
            if c[0] != 0:
                b = wsk[wsn - TAIL - 4 * (nq + 1) - 4:wsn - TAIL + 4].cpu().numpy().tobytes()
                n_miss = struct.unpack("<i", b[:4])[0]
                n_miss2, key = struct.unpack("<iI", b[-8:])
                u = (key & 0x7FFFFFFF) if key & 0x80000000 else (~key & 0xFFFFFFFF)
                fl = struct.unpack("<f", struct.pack("<I", u))[0] if key else float("nan")
                info[c] = f"floor {fl:.4f}, {n_miss} in the second pass, {n_miss2} after it"
    call("fwav_debug_topk_floor", -1, 0.0)
    for c in CONFIGS:
        name = {0: "off", -1: "default"}.get(int(c[0]), f"rank {int(c[1])}")
        print(f"{nq} queries, floor {name}: median {np.median(times[c]):.3f} ms  {info.get(c, '')}", flush=True)
    print(f"{nq} queries: all candidates identical={same}", flush=True)
