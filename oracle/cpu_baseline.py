"""CPU BASELINE — TEST/BENCH INFRASTRUCTURE ONLY (run as a child process of bench.py on rank 0).

Times the oracle restatement of the reference CPU path on a bounded sample of the bench workload and
extrapolates the full-run compress time the way BASELINE.md §4 prescribes:

    T = t_voiced+ranges+pool (full run) + nd · t_embed + max(nr_active · t_search / W, nr · t_affine)

with the reference's cost structure: per-domain scipy DCT embedding in one process (fractal.py:271-275),
per-range sgemv + argpartition in W search processes (fractal.py:1180-1207, 598-630) and a numpy batched
affine solve (B = 512) in one process running beside them (fractal.py:637-754).  W = the search processes: the
reference forks cpu_count()//2 (fractal.py:1180-1181), but the GPU box shows the whole machine's CPUs (256) while a
one-GPU job owns a 16-CPU share, so W is swept over 4/8/16 (capped at the share) and the fastest is reported, with
the sweep, the CPU model and the host copy bandwidth beside it.

Prints one JSON object on stdout.
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

import numpy as np
import scipy.fftpack
from threadpoolctl import threadpool_limits

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "audio-compression_amd"))

from oracle import fractal_oracle as O  # noqa: E402


def embed_rowwise(pool_rows: np.ndarray) -> np.ndarray:
    """multi_head_embedding per row (fractal.py:166-208, 154-164) — the reference's per-domain cost."""
    out = np.empty((len(pool_rows), 16), np.float32)
    for j, x in enumerate(pool_rows):
        x = np.asarray(x, np.float32)
        v = scipy.fftpack.dct(x, norm="ortho") * np.linspace(1.0, 2.0, len(x))
        take = min(8, max(0, len(v) - 1))
        e = np.zeros(8, np.float32)
        e[:take] = v[1:1 + take].astype(np.float32)
        n = np.linalg.norm(e)
        if n > 1e-8:
            e = e / n
        d = np.diff(x, prepend=x[0]) * np.linspace(1.0, 2.0, len(x))
        t = scipy.fftpack.dct(d, norm="ortho")[:8]
        nt = np.linalg.norm(t)
        if nt > 1e-8:
            t = t / nt
        out[j, :8] = e
        out[j, 8:8 + len(t)] = t.astype(np.float32)
        out[j, 8 + len(t):] = 0
    return out


_EMB = None


def _search_worker(args):
    rows, k = args
    with threadpool_limits(1):
        t0 = time.perf_counter()
        O.topk_candidates_loop(_EMB, np.asarray(rows), k)
        return time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--workers", default=None,
                    help="search processes, or a comma-separated sweep (default: the reference's cpu_count()//2 "
                         "capped at the box's CPU share, swept over 4/8/16)")
    ap.add_argument("--cpu-share", type=int, default=int(os.environ.get("FWAV_CPU_SHARE", "16")),
                    help="CPUs this job may use (the GPU box gives one GPU a 16-CPU share of a larger machine)")
    ap.add_argument("--search-sample", type=int, default=96, help="ranges per search process")
    ap.add_argument("--embed-sample", type=int, default=16384)
    ap.add_argument("--affine-sample", type=int, default=2048)
    args = ap.parse_args()
    from fwav import synth
    c = synth.CONFIGS[args.config]
    sig, sr, sw = synth.make_config_signal(args.config)
    tile, K = c["tile"], c["top_k"]
    rs, step = O.geometry(tile)

    t0 = time.perf_counter()
    vm = O.voiced_detection(sig, 2 * rs, 1e-4)
    ranges, _ = O.form_ranges(sig, vm, rs)
    pool = O.domain_pool(sig, tile, rs, step)
    t_pool = time.perf_counter() - t0
    nr, nd = len(ranges), len(pool)

    emb_full = O.embed(pool)  # fast batched restatement, only to give the search its full-size table
    rng = np.random.default_rng(0)
    sel = rng.choice(nd, size=min(args.embed_sample, nd), replace=False)
    with threadpool_limits(1):
        t0 = time.perf_counter()
        embed_rowwise(pool[sel])
        t_emb = (time.perf_counter() - t0) / len(sel)

    pruned = O.range_energy_pruned(ranges, 1e-4)
    act = np.nonzero(~pruned)[0]
    global _EMB
    _EMB = emb_full
    ref_w = max(1, (os.cpu_count() or 1) // 2)  # the reference forks cpu_count()//2 search workers (:1180-1181)
    if args.workers:
        Ws = sorted({max(1, int(w)) for w in str(args.workers).split(",")})
    else:
        Ws = sorted({w for w in (4, 8, 16, ref_w) if w <= max(1, args.cpu_share)} or {1})
    rows0 = rng.choice(act, size=max(8, args.search_sample // 4), replace=False)
    t0 = time.perf_counter()
    _search_worker((rows0, K))
    t_search_1 = (time.perf_counter() - t0) / max(8, args.search_sample // 4)
    ctx = mp.get_context("fork")
    sweep = {}
    for w in Ws:
        rows_w = [rng.choice(act, size=args.search_sample, replace=False) for _ in range(w)]
        t0 = time.perf_counter()
        with ctx.Pool(w) as p:
            p.map(_search_worker, [(r, K) for r in rows_w])
        sweep[w] = (time.perf_counter() - t0) / (w * args.search_sample)  # s per range with w processes
    W = min(sweep, key=sweep.get)
    t_search_w = sweep[W]

    arows = rng.choice(act, size=min(args.affine_sample, len(act)), replace=False)
    cand = O.topk_candidates(emb_full, nr, K, ~np.isin(np.arange(nr), arows))[0][arows]
    with threadpool_limits(1):
        t0 = time.perf_counter()
        for s in range(0, len(arows), 512):
            O.affine(ranges[arows[s:s + 512]], cand[s:s + 512], pool)
        t_aff = (time.perf_counter() - t0) / len(arows)

    T = t_pool + nd * t_emb + max(len(act) * t_search_w, nr * t_aff)
    sample = (f"{args.config}: full voiced+ranges+pool; embed {len(sel)} domains rowwise; search "
              f"{W}x{args.search_sample} ranges vs the full {nd}-domain table in {W} processes (best of a sweep "
              f"over {Ws} processes; the reference would fork cpu_count()//2 = {ref_w}"
              f"{', capped at this job' + chr(39) + f's {args.cpu_share}-CPU share' if ref_w > args.cpu_share else ''}); affine {len(arows)} ranges; extrapolated to {nr} ranges")
    print(json.dumps(dict(value=nr / T, unit="ranges/s", cores=W, kind="port", sample=sample, extrapolated=True,
                          t_total_s=T, t_pool_s=t_pool, t_embed_per_domain_s=t_emb,
                          t_search_per_range_1proc_s=t_search_1, t_search_per_range_Wproc_s=t_search_w,
                          search_sweep_s_per_range={str(k): v for k, v in sweep.items()},
                          reference_workers=ref_w, cpu_share=args.cpu_share,
                          t_affine_per_range_s=t_aff, n_ranges=nr, n_domains=nd, cpu_count=os.cpu_count(),
                          cpu_model=cpu_model(), host_copy_gbs=host_copy_gbs())))


def cpu_model() -> str:
    """The lscpu "Model name" (read from /proc/cpuinfo, which lscpu reports)."""
    try:
        for line in open("/proc/cpuinfo"):
            if line.lower().startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def host_copy_gbs(mb: int = 512, reps: int = 5) -> float:
    """STREAM-style copy bandwidth of one host thread: (read + write bytes) / time, best of `reps`."""
    a = np.ones(mb * (1 << 20) // 4, np.float32)
    b = np.empty_like(a)
    best = float("inf")
    for _ in range(reps):
        t0 = time.perf_counter()
        np.copyto(b, a)
        best = min(best, time.perf_counter() - t0)
    return 2 * a.nbytes / best / 1e9


if __name__ == "__main__":
    main()
