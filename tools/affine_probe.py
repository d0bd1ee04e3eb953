#!/usr/bin/env python3
"""Affine solver at cfg4 scale (diagnostic): where do its rows come from and what bounds it?

Builds the cfg4 signal (60 min, 48 kHz: 86.4 M domains, a 2.76 GB pool), searches the first --queries ranges
against the whole table, then times fwav_affine (HIP events around the launch only) on those real candidates:
  warm  : back to back (the rows the candidates touch stay in L2 / the Infinity Cache between launches)
  cold  : a 1 GiB buffer is rewritten before every launch, so the pool rows come from HBM (the pipeline's case:
          the search streams the whole fp16 table right before the affine solve)
  prefix: candidates folded into the first 2^20 rows (32 MB of pool; an L2/MALL-resident bound)
usage: python tools/affine_probe.py [--queries N] [--only warm,cold,prefix] [--lib path/to/libfwav.so ...]
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "audio-compression_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--queries", type=int, default=262_144)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default="warm,cold,prefix")
    ap.add_argument("--lib", action="append", default=[])
    a = ap.parse_args()
    import __graft_entry__
    __graft_entry__.build()
    from fwav import engine, synth
    from fwav._lib import SIGNATURES, call
    dev = torch.device("cuda", 0)
    sig_h, _, _ = synth.make_config_signal("cfg4")
    sig = torch.from_numpy(sig_h).to(dev)
    K, q = 64, a.queries
    res = engine.compress_device(sig, 2048, K, shard=(0, q), keep_intermediates=True)
    torch.cuda.synchronize()
    nd, rs = res.n_domains, res.range_size
    libs = [("default", None)]
    for p in a.lib:
        L = C.CDLL(os.path.abspath(p))
        r_, args_ = SIGNATURES["fwav_affine"]
        L.fwav_affine.restype, L.fwav_affine.argtypes = r_, args_
        libs.append((os.path.basename(p), L))
    st = torch.cuda.current_stream(dev)
    flush = torch.empty(1 << 28, dtype=torch.float32, device=dev)  # 1 GiB
    cand_real = res.cand[:q * K].clone()
    cand_prefix = torch.where(cand_real >= 0, cand_real % (1 << 20), cand_real)
    nbytes = q * (4 * rs + 4 * K + 4 * K * rs + 17)
    out = {"queries": q, "n_domains": nd, "bytes_per_launch": nbytes}
    # candidate locality: rows shared by consecutive ranges, distinct 64-B sectors per range and per 256 ranges
    import numpy as np
    c = cand_real[:4096 * K].view(4096, K).cpu().numpy()
    out["overlap_i_i1"] = float(np.mean([len(set(c[i]) & set(c[i + 1])) for i in range(4095)]))
    out["sectors64_per_range"] = float(np.mean([len(np.unique(r // 2)) for r in c]))
    out["sectors64_per_256_ranges_per_range"] = float(np.mean([len(np.unique(c[i:i + 256] // 2)) / 256
                                                               for i in range(0, 4096, 256)]))
    print(json.dumps(out), flush=True)
    ref = None
    for lname, L in libs:
        for mode in a.only.split(","):
            cand = cand_prefix if mode == "prefix" else cand_real
            o = [torch.empty(q, dtype=dt, device=dev) for dt in (torch.int32, torch.float32, torch.float32,
                                                                  torch.uint8, torch.float32)]
            args = (res.ranges.data_ptr(), q, rs, cand.data_ptr(), K, res.pool.data_ptr(), nd, 16.0,
                    *[t.data_ptr() for t in o], st.cuda_stream)
            fn = (lambda: call("fwav_affine", *args)) if L is None else (lambda: L.fwav_affine(*args))
            fn()
            ms = []
            for _ in range(a.reps):
                if mode == "cold":
                    flush.fill_(1.0)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                fn()
                e1.record(st)
                torch.cuda.synchronize(dev)
                ms.append(e0.elapsed_time(e1))
            ms.sort()
            med = ms[len(ms) // 2]
            same = None
            if mode != "prefix":
                cur = torch.cat([t.view(torch.uint8).view(-1) for t in o])
                if ref is None:
                    ref = cur
                same = bool(torch.equal(cur, ref))
            out[f"{lname}:{mode}"] = {"median_ms": med, "min_ms": ms[0], "alg_gbs": nbytes / (med * 1e-3) / 1e9,
                                      "hbm_frac": nbytes / (med * 1e-3) / 8e12, "identical": same}
            print(lname, mode, json.dumps(out[f"{lname}:{mode}"]), flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
