"""Diagnostic: a stream of deferred compress calls on cfg2 / cfg3 — wall time per call with the host tie work
overlapped (defer_ties) vs synchronous, with fwav.ties' phase trace.  usage: FWAV_TIES_TRACE=1 python tools/diag/ties_defer.py cfg3"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "audio-compression_amd")]
import torch

from fwav import engine, synth

name = sys.argv[1]
cfg = synth.CONFIGS[name]
sig = torch.from_numpy(synth.make_config_signal(name, seed=0)[0]).cuda()
for defer in (False, True):
    r = engine.compress_device(sig, cfg["tile"], cfg["top_k"], defer_ties=defer)
    r.wait()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rs = [engine.compress_device(sig, cfg["tile"], cfg["top_k"], defer_ties=defer) for _ in range(4)]
    t1 = time.perf_counter()
    for r in rs:
        r.wait()
    torch.cuda.synchronize()
    print(f"{name} defer={defer}: {(time.perf_counter() - t0) / 4 * 1e3:.1f} ms per call (launch loop "
          f"{(t1 - t0) * 1e3:.1f} ms), n_resolved {rs[-1].n_resolved}", flush=True)
