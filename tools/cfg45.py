#!/usr/bin/env python3
"""cfg4 / cfg5 measurements on ONE GPU (diagnostic; prints one JSON line).

cfg4 per GPU: the 60 min 48 kHz signal (172.8 M samples, 21.6 M ranges, 86.4 M domains) is built on the device
(voiced, pool, embeddings for the whole table) and the first --queries ranges — one rank's share of an 8-way
shard is 2.7 M — are searched against the FULL 86.4 M-domain table and solved, with per-stage HIP events.

cfg5: the decode of a cfg4-sized match set (21.6 M ranges) over the cfg4 pool: defaults (8 iterations, eps 1e-3)
and forced 50 iterations (eps 0).  The matches of the searched ranges are real; the rest are drawn at random
(decode time does not depend on the values).  With --check, the forced-50 reconstruction of the first
--check-ranges ranges is compared bit-for-bit with the oracle (ranges are independent when no early exit occurs).
"""
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

F16_PEAK = 2516.6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--queries", type=int, default=337_500)
    ap.add_argument("--reps", type=int, default=1)
    ap.add_argument("--seconds", type=float, default=3600.0)
    ap.add_argument("--no-decode", action="store_true")
    ap.add_argument("--check", action="store_true")
    ap.add_argument("--check-ranges", type=int, default=100_000)
    a = ap.parse_args()
    import __graft_entry__
    __graft_entry__.build()
    from fwav import engine, synth
    dev = torch.device("cuda", 0)
    t0 = time.perf_counter()
    sig_h, sr, _ = synth.make_config_signal("cfg4", seconds=a.seconds, seed=0)
    t_gen = time.perf_counter() - t0
    sig = torch.from_numpy(sig_h).to(dev)
    out = {"config": "cfg4", "samples": int(sig_h.size), "t_signal_gen_s": t_gen}
    q = a.queries
    res = None
    for rep in range(a.reps):
        ev = {}
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        res = engine.compress_device(sig, 2048, 64, energy_thresh=1e-4, shard=(0, q), events=ev)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t1
        st = {k: v[0].elapsed_time(v[1]) for k, v in ev.items()}
        na = int(res.n_active.item())
        fl = 2.0 * na * res.n_domains * 16
        out[f"rep{rep}"] = {"wall_s": wall, "stage_ms": st, "active_queries": na, "n_ties": res.n_ties,
                            "n_resolved": res.n_resolved,
                            "sim_topk_tflops": fl / (st["sim_topk"] * 1e-3) / 1e12,
                            "sim_topk_frac_f16_peak": fl / (st["sim_topk"] * 1e-3) / 1e12 / F16_PEAK,
                            "full_cfg4_search_s_extrapolated": st["sim_topk"] * 1e-3 * res.n_ranges / q}
    out.update(n_ranges=res.n_ranges, n_domains=res.n_domains, queries=q)
    if not a.no_decode:
        nr, rs, nd = res.n_ranges, res.range_size, res.n_domains
        g = torch.Generator(device=dev)
        g.manual_seed(5)
        idx = torch.randint(0, nd, (nr,), device=dev, generator=g, dtype=torch.int32)
        s = (torch.rand(nr, device=dev, generator=g) * 2 - 1).to(torch.float32)
        o = (torch.randn(nr, device=dev, generator=g) * 0.05).to(torch.float32)
        sym = (torch.rand(nr, device=dev, generator=g) < 0.5).to(torch.uint8)
        idx[:q], s[:q], o[:q], sym[:q] = res.idx, res.s, res.o, res.sym
        dec = {}
        for name, iters, eps in (("default", 8, 1e-3), ("forced50", 50, 0.0)):
            engine.decompress_device(idx, s, o, sym, res.pool, nr, rs, iters, eps)
            torch.cuda.synchronize()
            reps = 3
            td = time.perf_counter()
            for _ in range(reps):
                rec, ran, deltas = engine.decompress_device(idx, s, o, sym, res.pool, nr, rs, iters, eps)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - td) / reps
            dec[name] = {"iterations": ran, "ms": dt * 1e3, "range_iterations_per_s": nr * ran / dt,
                         "streaming_equivalent_gbs": nr * (12 * rs + 17) * ran / dt / 1e9,
                         "first_deltas": deltas[:3]}
            if name == "forced50" and a.check:
                from oracle import fractal_oracle as O
                m = a.check_ranges
                pool_h = res.pool.view(nd, rs)
                ih = idx[:m].cpu().numpy()
                used = np.unique(ih[ih >= 0])
                # the oracle only needs the rows these ranges use: remap them into a compact pool
                sub = pool_h[torch.from_numpy(used).to(dev).long()].cpu().numpy()
                remap = np.searchsorted(used, np.maximum(ih, 0)).astype(np.int32)
                remap[ih < 0] = -1
                ref, it, _ = O.decode(remap, s[:m].cpu().numpy(), o[:m].cpu().numpy(), sym[:m].cpu().numpy(), sub,
                                      m, rs, iterations=50, convergence_eps=0.0)
                dec[name]["check_ranges"] = m
                dec[name]["bit_exact_vs_oracle"] = bool(np.array_equal(
                    rec[:m * rs].cpu().numpy().view(np.uint32), ref.view(np.uint32))) and it == 50
        out["decode_cfg5"] = dec
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
