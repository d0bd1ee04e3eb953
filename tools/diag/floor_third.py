#!/usr/bin/env python3
"""How often does the speculative floor's second pass cut a query (a cold third pass)?  For several signals and every
rank share of N = 1, 2, 4, 8, one product compress per share (keep_intermediates), reading the search workspace
(fwav_debug_sim_topk_layout): the first floor, the second floor, the misses of the first and second pass.
usage: python tools/diag/floor_third.py [--seeds 0 1 2]"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "audio-compression_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def key2f(k: int) -> float:
    k &= 0xFFFFFFFF
    if k == 0:
        return float("nan")
    u = (k & 0x7FFFFFFF) if (k & 0x80000000) else (~k & 0xFFFFFFFF)
    return float(np.array([u], np.uint32).view(np.float32)[0])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, nargs="+", default=[0, 1, 2])
    a = ap.parse_args()
    import __graft_entry__
    __graft_entry__.build()
    from fwav import dist as fdist
    from fwav import engine, synth
    from fwav._lib import sim_topk_layout
    dev = torch.device("cuda", 0)
    thirds = 0
    cases = 0
    for seed in a.seeds:
        for name, sig_h in (("noise", synth.noise(60.0, 44100, seed=seed)),
                            ("speech", synth.speech_like(60.0, 44100, seed=seed))):
            sig = torch.from_numpy(sig_h).to(dev)
            rg, nr_, rs_ = engine.ranges_device(sig, 2048, 1e-4)
            for N in (1, 2, 4, 8):
                blocks = fdist.prune_balanced_bounds(rg, nr_, rs_, 1e-4, N)
                row = []
                for shard in blocks:
                    r = engine.compress_device(sig, 2048, 64, energy_thresh=1e-4, shard=shard,
                                               keep_intermediates=True)
                    torch.cuda.synchronize()
                    if r.search_ws is None:
                        row.append("sliced")
                        continue
                    lay = sim_topk_layout(r.shard[1] - r.shard[0], r.n_domains)
                    w = r.search_ws
                    i32 = lambda off: int(w[off:off + 4].view(torch.int32).item())  # noqa: E731
                    fk = w[lay["floor_key"]:lay["floor_key"] + 8].view(torch.int32).cpu().numpy()
                    f1, f2 = key2f(int(fk[0])), key2f(int(fk[1]))
                    m1, m2 = i32(lay["n_miss"]), i32(lay["n_miss2"])
                    cases += 1
                    thirds += m2 > 0
                    # the queries' K-th scores (the 64th candidate's score, f32 dot): how far below the pilots' smallest
                    # estimate (f2 + 0.15) the lowest ones lie
                    na = int(r.n_active.item())
                    act = r.active[:na].long()
                    c = r.cand.view(-1, 64)[act, 63].long()
                    lo = r.shard[0]
                    kth = (r.emb.view(-1, 16)[act + lo] * r.emb.view(-1, 16)[c]).sum(1)
                    low = torch.sort(kth).values[:3].tolist()
                    row.append(f"{na}a f={f1:.3f}/{f2:.3f} miss {m1}/{m2} kth_min {low[0]:.3f},{low[1]:.3f},{low[2]:.3f} "
                               f"gap {f2 + 0.15 - low[0]:.3f}")
                print(f"{name} seed {seed} N={N}: " + "; ".join(row), flush=True)
    print(f"third passes: {thirds} of {cases} searches", flush=True)


if __name__ == "__main__":
    main()
