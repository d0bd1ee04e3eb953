"""A/B the batched affine solve of several libfwav builds on REAL candidates at cfg4 scale (the 2.76 GB pool is ten
times the 256 MB Infinity Cache, so row gathers are HBM traffic) and on uniformly random candidates.
usage: python tools/ab_affine.py lib1.so lib2.so ...   [AB_Q=262144 ranges searched for their candidates]"""
import ctypes as C
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "audio-compression_amd")]
import torch

import __graft_entry__

__graft_entry__.build()
from fwav import engine, synth  # noqa: E402
from fwav._lib import SIGNATURES  # noqa: E402

q = int(os.environ.get("AB_Q", 262144))
sig_h, _, _ = synth.make_config_signal("cfg4")
sig = torch.from_numpy(sig_h).cuda()
res = engine.compress_device(sig, 2048, 64, shard=(0, q), keep_intermediates=True)
torch.cuda.synchronize()
nd, rs, K = res.n_domains, res.range_size, 64
ranges = res.ranges[:q * rs]
cands = {"real": res.cand[:q * K].clone(),
         "random": torch.randint(0, nd, (q * K,), device="cuda", dtype=torch.int32)}
nbytes = q * (4 * rs + 4 * K + 4 * K * rs + 17)
st = torch.cuda.current_stream().cuda_stream
for path in sys.argv[1:]:
    L = C.CDLL(os.path.abspath(path))
    r_, a_ = SIGNATURES["fwav_affine"]
    L.fwav_affine.restype, L.fwav_affine.argtypes = r_, a_
    for name, cand in cands.items():
        out = [torch.empty(q, dtype=dt, device="cuda") for dt in (torch.int32, torch.float32, torch.float32,
                                                                    torch.uint8, torch.float32)]
        args = (ranges.data_ptr(), q, rs, cand.data_ptr(), K, res.pool.data_ptr(), nd, 16.0,
                *[t.data_ptr() for t in out], st)
        assert L.fwav_affine(*args) == 0
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            L.fwav_affine(*args)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        same = bool(torch.equal(out[0], res.idx[:q])) if name == "real" else None
        print(f"{os.path.basename(path):24s} {name:6s} {ms:.3f} ms  {nbytes / ms / 1e6:.0f} GB/s  "
              f"{nbytes / ms / 1e6 / 8000:.3f} of 8 TB/s  idx==pipeline: {same}", flush=True)
