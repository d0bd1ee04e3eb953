"""Timing (tools only): consecutive cfg2 compress steps (deferred ties, as bench.py's timed loop) issued on 1, 2 or 3
HIP streams in turn, so that one step's search tail can overlap the next step's kernels.
usage: python tools/streams_ab.py [steps]"""
import os
import sys
import time

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "audio-compression_amd")]
import torch

import __graft_entry__

__graft_entry__.build()
from fwav import engine, synth  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)
sig = torch.from_numpy(synth.make_config_signal("cfg2", seed=0)[0]).to(dev)
torch.cuda.synchronize()
for rnd in range(2):
    for ns in (1, 2, 3):
        streams = [torch.cuda.Stream(dev) for _ in range(ns)]
        for s_ in streams:
            s_.wait_stream(torch.cuda.current_stream(dev))
        pend = []

        def run(n):
            for i in range(n):
                with torch.cuda.stream(streams[i % ns]):
                    pend.append(engine.compress_device(sig, 2048, 64, energy_thresh=1e-4, defer_ties=True))
            for r in pend:
                r.wait()
            pend.clear()
        run(3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run(K)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / K * 1e3
        print(f"round {rnd} streams {ns}: {dt:.2f} ms per step, {330750 / dt * 1e3 / 1e6:.2f} M ranges/s", flush=True)
