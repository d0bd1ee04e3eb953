#!/usr/bin/env python3
"""One rank's share of the sharded cfg2 compress, on one GPU (diagnostic for strong scaling): the step time of
compress_device(sig, shard=block r of N) for N = 1, 2, 4, 8 and every rank r — everything a rank of bench.py --gpus N
does except the collectives — with per-stage HIP events and the host wall time per step, ties resolved synchronously
("sync") and deferred with two calls in flight as bench.py's timed loop runs them ("pipelined").  The slowest rank
sets the step time.
usage: python tools/shard_step.py [--steps 20]"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "audio-compression_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--ns", default="1,2,4,8", help="world sizes to simulate")
    ap.add_argument("--ranks", default="", help="only these ranks (comma list; default every rank)")
    ap.add_argument("--lags", default="3", help="calls in flight for the pipelined loop (comma list: one column each)")
    ap.add_argument("--tie-order", default="numpy", help="compress_device tie_order (index: no host tie step)")
    ap.add_argument("--streams", type=int, default=1,
                    help="pipelined loop: consecutive calls alternate over this many HIP streams")
    a = ap.parse_args()
    lags = [int(x) for x in a.lags.split(",")]
    import __graft_entry__
    __graft_entry__.build()
    from fwav import dist as fdist
    from fwav import engine, synth
    dev = torch.device("cuda", 0)
    cfg = synth.CONFIGS[a.config]
    sig_h, _, _ = synth.make_config_signal(a.config, seed=0)
    sig = torch.from_numpy(sig_h).to(dev)
    tile, K = cfg["tile"], cfg["top_k"]
    out = {}
    for N in [int(x) for x in a.ns.split(",")]:
        per = []
        rg, nr_, rs_ = engine.ranges_device(sig, tile, 1e-4)
        blocks = fdist.prune_balanced_bounds(rg, nr_, rs_, 1e-4, N)
        for rank in ([int(x) for x in a.ranks.split(",") if int(x) < N] if a.ranks else range(N)):
            # the bench computes these bounds every step on a side stream, off the critical path (fwav.dist); here
            # they are computed once, so that the timed loop has no host synchronisation either
            shard = blocks[rank]
            for _ in range(2):
                engine.compress_device(sig, tile, K, energy_thresh=1e-4, shard=shard, tie_order=a.tie_order)
            torch.cuda.synchronize()
            evs = []
            t0 = time.perf_counter()
            for _ in range(a.steps):
                ev = {}
                r = engine.compress_device(sig, tile, K, energy_thresh=1e-4, shard=shard, events=ev,
                                           tie_order=a.tie_order)
                evs.append(ev)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) / a.steps * 1e3
            st = {k: float(np.mean([e[k][0].elapsed_time(e[k][1]) for e in evs])) for k in evs[0]}
            pipes = {}
            streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(a.streams - 1)]
            host = {}
            for lag in lags:
                inflight = []
                t_call = t_wait = 0.0
                t0 = time.perf_counter()
                for i in range(a.steps):
                    ta = time.perf_counter()
                    with torch.cuda.stream(streams[i % len(streams)]):
                        inflight.append(engine.compress_device(sig, tile, K, energy_thresh=1e-4, shard=shard,
                                                               defer_ties=True, tie_order=a.tie_order))
                    tb = time.perf_counter()
                    while len(inflight) > lag:  # calls in flight (bench.py: 3)
                        inflight.pop(0).wait()
                    t_call += tb - ta
                    t_wait += time.perf_counter() - tb
                for x in inflight:
                    x.wait()
                torch.cuda.synchronize()
                pipes[lag] = (time.perf_counter() - t0) / a.steps * 1e3
                # host ms per call inside compress_device (launch + any host synchronisation) and blocked in wait()
                host[lag] = {"call_ms": t_call / a.steps * 1e3, "wait_ms": t_wait / a.steps * 1e3}
            pipe = pipes[lags[0]]
            per.append({"rank": rank, "ranges": r.shard[1] - r.shard[0], "tie_rows": r.n_resolved,
                        "wall_ms_sync": wall, "wall_ms_pipelined": pipe,
                        "wall_ms_pipelined_by_lag": pipes, "host_by_lag": host, "stage_ms": st})
        out[N] = {"max_wall_ms_sync": max(p["wall_ms_sync"] for p in per),
                  "max_wall_ms_pipelined": max(p["wall_ms_pipelined"] for p in per), "ranks": per}
        print(N, json.dumps(out[N]), flush=True)
    if 1 in out:
        print(json.dumps({N: {"speedup_sync": out[1]["max_wall_ms_sync"] / v["max_wall_ms_sync"],
                              "speedup_pipelined": out[1]["max_wall_ms_pipelined"] / v["max_wall_ms_pipelined"]}
                          for N, v in out.items()}), flush=True)

if __name__ == "__main__":
    main()
