#!/usr/bin/env python3
"""Do the speculative floor's misses cluster?  After one product compress (cfg2 and a speech-like signal), read the
first pass's miss list from the search workspace and count, per miss q, whether its neighbours q ± s (s = 1, 2) were
misses too: a neighbour that was not (an active query the first pass emitted) holds a final top K whose shifted
domains bound q's K-th score from below (neighbour seeds).  Also prints the queries' K-th exact scores
against the pilots' floors (from the candidate rows: exact f32 scores of the K-th candidate).
usage: python tools/diag/miss_neighbours.py"""
from __future__ import annotations

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "audio-compression_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def key2f(k: int) -> float:
    u = (k & 0x7FFFFFFF) if (k & 0x80000000) else (~k & 0xFFFFFFFF)
    return float(np.array([u], np.uint32).view(np.float32)[0])


def main():
    import __graft_entry__
    __graft_entry__.build()
    from fwav import engine, synth
    from fwav._lib import sim_topk_layout
    for name, sig_h in (("cfg2", synth.make_config_signal("cfg2")[0]), ("speech60", synth.speech_like(60.0, 44100, seed=0))):
        sig = torch.from_numpy(sig_h).cuda()
        r = engine.compress_device(sig, 2048, 64, keep_intermediates=True)
        torch.cuda.synchronize()
        lay = sim_topk_layout(r.n_ranges, r.n_domains)
        ws = r.search_ws
        i32 = lambda off, n: ws[off:off + 4 * n].view(torch.int32).cpu().numpy()  # noqa: E731
        n_miss = int(i32(lay["n_miss"], 1)[0])
        miss = np.sort(i32(lay["miss"], n_miss))
        fk = ws[lay["floor_key"]:lay["floor_key"] + 8].view(torch.int32).cpu().numpy().astype(np.int64) & 0xFFFFFFFF
        nact = int(r.n_active.item())
        act = r.active[:nact].cpu().numpy() if hasattr(r, "active") else np.arange(r.n_ranges)
        ism = np.zeros(r.n_ranges + 4, bool)
        ism[miss] = True
        isact = np.zeros(r.n_ranges + 4, bool)
        isact[act] = True
        out = [f"{name}: {r.n_ranges} ranges, {nact} active, {n_miss} misses; floor {key2f(int(fk[0])):.4f}, second "
               f"floor {key2f(int(fk[1])):.4f}"]
        for s in (1, 2):
            good = np.zeros(n_miss, bool)
            for sh in (-s, s):
                nb = miss + sh
                ok = (nb >= 0) & (nb < r.n_ranges)
                g = np.zeros(n_miss, bool)
                g[ok] = isact[nb[ok]] & ~ism[nb[ok]]
                good |= g
            out.append(f"  misses with an emitted neighbour within ±{s}: {good.sum()} ({100.0 * good.mean():.1f} %)")
        # run lengths of consecutive misses
        if n_miss:
            runs = np.diff(np.flatnonzero(np.diff(np.r_[-10, miss.astype(np.int64), 1 << 40]) != 1))
            out.append(f"  runs of consecutive misses: {len(runs)}, mean length {runs.mean():.2f}, max {runs.max()}")
        print("\n".join(out), flush=True)


if __name__ == "__main__":
    main()
