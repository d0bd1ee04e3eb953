#!/usr/bin/env python3
"""Repeated fwav_sim_topk calls of one configuration through the DEBUG library, so that its process-global knobs
apply (FWAV_DEBUG_TOPK_FLOOR="mode[:value]", FWAV_DEBUG_TOPK_GEOMETRY, FWAV_DEBUG_TOPK_P2): a target for
`rocprofv3 --kernel-trace --stats` per knob setting.  Prints the median call time (HIP events) and the floor's
miss counts of the last call.
usage: [AB_NQ=41344] [AB_LO=first query] [AB_TIES=1] [AB_PLAN=rt,P] [AB_RUNS=1 | AB_ENGINE_ACTIVE=1] python tools/diag/topk_reps.py [reps]"""
from __future__ import annotations

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "audio-compression_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 9
    import __graft_entry__
    __graft_entry__.build()
    from fwav import engine, synth
    from fwav.nporder import blas_threads
    from fwav._lib import debug_lib, sim_topk_layout
    d = debug_lib()
    sig = torch.from_numpy(synth.noise(60.0, 44100)).cuda()
    r = engine.compress_device(sig, 2048, 64, keep_intermediates=True)
    torch.cuda.synchronize()
    nd, nr = r.n_domains, r.n_ranges
    st = torch.cuda.current_stream().cuda_stream
    emb16 = torch.empty(2 * ((nd + 255) // 256) * 256 * 16, dtype=torch.float16, device="cuda")
    assert d.fwav_emb16_from_emb(r.emb.data_ptr(), nd, emb16.data_ptr(), st) == 0
    if os.environ.get("AB_PLAN"):  # "rt,pieces": the work-plan override (fwav_debug_topk_plan), before sizing
        assert d.fwav_debug_topk_plan(*[int(x) for x in os.environ["AB_PLAN"].split(",")]) == 0
    nq = int(os.environ.get("AB_NQ", nr))
    # the last rank's block (bench.py's roofline_rank_share), or the block at AB_LO
    lo = int(os.environ["AB_LO"]) if os.environ.get("AB_LO") else nr - nq
    active = torch.arange(nq, dtype=torch.int32, device="cuda")  # (cfg2 noise: every range active)
    if os.environ.get("AB_RUNS") == "1":  # fwav_prune's order: runs of 64 consecutive ranges in a random run order
        g = torch.Generator().manual_seed(0)
        runs = torch.randperm((nq + 63) // 64, generator=g)
        active = torch.cat([torch.arange(r * 64, min(nq, r * 64 + 64), dtype=torch.int32) for r in runs.tolist()]).cuda()
    elif os.environ.get("AB_ENGINE_ACTIVE") == "1":  # the product's own active list of this block
        rb = engine.compress_device(sig, 2048, 64, shard=(nr - nq, nr), keep_intermediates=True)
        torch.cuda.synchronize()
        active = rb.active[:int(rb.n_active.item())].clone()
        assert active.numel() == nq
    n_active = torch.tensor([nq], dtype=torch.int32, device="cuda")
    wsn = d.fwav_sim_topk_workspace_size(nq, nd, 64)
    wsk = torch.empty(wsn, dtype=torch.uint8, device="cuda")
    cand = torch.empty(nq * 64, dtype=torch.int32, device="cuda")
    # AB_TIES=1: the search also lists its tied queries (the product's tie_order="numpy" calls pass this list)
    ties = (torch.empty(d.fwav_tie_list_size(nq), dtype=torch.int32, device="cuda")
            if os.environ.get("AB_TIES") == "1" else None)
    ms = []
    for i in range(reps + 1):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        rc = d.fwav_sim_topk(r.emb.data_ptr(), emb16.data_ptr(), nd, active.data_ptr(), n_active.data_ptr(), nq, lo,
                             64, blas_threads(), cand.data_ptr(), None if ties is None else ties.data_ptr(), wsk.data_ptr(),
                             wsn, st)
        e1.record()
        torch.cuda.synchronize()
        assert rc == 0
        if i:
            ms.append(e0.elapsed_time(e1))
    lay = sim_topk_layout(nq, nd)
    cnt = lambda k: int(wsk[lay[k]:lay[k] + 4].view(torch.int32).item())  # noqa: E731
    ref = r.cand.view(-1, 64)[lo:].reshape(-1)
    same = bool(torch.equal(cand, ref)) if r.n_resolved == 0 else None
    print(f"{nq} queries: median {np.median(ms):.3f} ms (min {min(ms):.3f}); floor misses {cnt('n_miss')} / "
          f"{cnt('n_miss2')}; env floor={os.environ.get('FWAV_DEBUG_TOPK_FLOOR', '-')} "
          f"geometry={os.environ.get('FWAV_DEBUG_TOPK_GEOMETRY', '-')} plan={os.environ.get('AB_PLAN', '-')}; equal to the product rows: {same}"
          + (f"; tied queries {int(ties[0].item())}" if ties is not None else ""), flush=True)


if __name__ == "__main__":
    main()
