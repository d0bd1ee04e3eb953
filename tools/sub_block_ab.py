"""Timing (tools only): compress_device with the search in one launch (sub_blocks=1: every tied row ranked by numpy
after the search) against the default sub-blocked search (tied rows of one slice ranked while the next searches), on
cfg3 (whole signal) and one rank's eighth of cfg4; outputs must be identical.
usage: python tools/sub_block_ab.py [cfg3|cfg4 ...]"""
import json
import os
import sys
import time

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "audio-compression_amd")]
import torch

import __graft_entry__

__graft_entry__.build()
from fwav import dist as fdist  # noqa: E402
from fwav import engine, synth  # noqa: E402

for cfg in sys.argv[1:] or ["cfg3", "cfg4"]:
    c = synth.CONFIGS[cfg]
    sig = torch.from_numpy(synth.make_config_signal(cfg, seed=0)[0]).cuda()
    shard = None
    if cfg == "cfg4":
        def shard(ranges, n_ranges, range_size):
            return fdist.prune_balanced_bounds(ranges, n_ranges, range_size, 1e-4, 8)[0]
    out = {}
    ref = None
    seen = set()

    def key_seen(x):
        if x in seen:
            return True
        seen.add(x)
        return False
    for nsub in (None, 1, None, 1):  # second round: staging slots already allocated
        ev = {}
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = engine.compress_device(sig, c["tile"], c["top_k"], energy_thresh=1e-4, shard=shard, sub_blocks=nsub,
                                   events=ev)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        st = {k: ev[k][0].elapsed_time(ev[k][1]) for k in ev}
        key = ("default" if nsub is None else f"sub_blocks={nsub}") + (" (again)" if key_seen(nsub) else "")
        out[key] = {"wall_s": wall, "stage_ms": st, "n_ties": r.n_ties, "n_resolved": r.n_resolved,
                    "sub_blocks": engine._tie_sub_blocks(r.shard[1] - r.shard[0], r.n_domains) if nsub is None else 1}
        outs = [t.cpu() for t in (r.idx, r.s, r.o, r.sym, r.err)]
        if ref is None:
            ref = outs
        else:
            out[key]["identical"] = all(torch.equal(a.view(torch.uint8), b.view(torch.uint8)) for a, b in zip(outs, ref))
        print(cfg, key, json.dumps(out[key]), flush=True)
        del r
