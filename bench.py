#!/usr/bin/env python3
"""Benchmark: ranges matched/sec at tile_size=2048, top-K=64 (BASELINE.json metric) on MI355X.

One step = one full compress hot path over ONE 60 s 44.1 kHz noise signal (cfg2, BASELINE.json configs[1]):
voiced detection → ranges → domain pool → embeddings → energy prune → similarity top-64 → affine solve with
mirror, all on device; the signal is resident in HBM before the timed region and the match arrays stay there.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N) runs the north star's sharded
path on the same single signal (strong scaling, "scaling": "strong"): rank 0 holds the signal in HBM, RCCL
broadcasts it over xGMI, every rank rebuilds ranges/pool/embeddings, searches + solves its prune-balanced block of
ranges, and the match arrays are gathered to rank 0 (fwav.dist.compress_sharded_start/finish).  The timed steps
include every broadcast and gather; up to three calls are in flight, so a call's host tie ranking (defer_ties, as
at N = 1) overlaps the next calls' searches before its gather; value = n_ranges / max-over-ranks step time.  N = 1
is the same path with no collective (compress_device), so the driver's per-N values form a strong-scaling curve.

Also reported: the dominant kernel's roofline (similarity top-K vs the fp16 MFMA peak; HIP events on the launch
stream; `traffic` = PMC bytes from a committed rocprofv3 pass of the same config, labelled with its source), the
affine solver's HBM roofline measured on a pool above the 256 MB MALL (the north star's ≥60 % target), per-stage
times, the decode (default and forced 50 iterations) and the CPU baseline (oracle restatement on this host,
bounded sample, rank 0 at N=1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "audio-compression_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md chip table (spec)
F16_MFMA_PEAK_TF = 2516.6    # dense f16 MFMA peak: v_mfma_f32_32x32x16_f16, 32 cycles/SIMD, 1024 SIMDs, 2.4 GHz
STAGES = ["voiced_ranges", "pool_embed", "prune", "sim_topk", "affine"]
WORKLOAD_TEXT = {"cfg1": "1 s 16 kHz mono sine sweep", "cfg2": "60 s 44.1 kHz mono white noise",
                 "cfg3": "10 min 44.1 kHz mono speech-like synthetic", "cfg4": "60 min 48 kHz mono white noise"}
TOPK_KERNEL = "k_sim_topk_f16"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--seconds", type=float, default=None, help="override signal length (debug)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="only the timed steps (profiling passes)")
    ap.add_argument("--cpu-workers", default=None, help="CPU baseline search processes (default: sweep)")
    ap.add_argument("--tie-order", default="numpy",
                    help="compress_device tie_order (diagnostic: 'index' drops the host ranking of exactly tied rows, "
                         "so matches may differ from the reference's where numpy's order among equal scores decides)")
    ap.add_argument("--streams", type=int, default=2,
                    help="HIP streams that consecutive timed calls alternate over (a call's kernels stay on one); "
                         "the same default at every N, so that the driver's 1 -> N curve compares like with like")
    return ap.parse_args()


def pmc_traffic(config: str):
    """HBM bytes per top-K launch from the committed PMC pass of THIS config (profiles/pmc_<config>.json, written by
    tools/pmc_summary.py from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of this bench), else None."""
    path = os.path.join(ROOT, "profiles", f"pmc_{config}.json")
    if not os.path.exists(path):
        return None, None
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    if d.get("config") != config:
        return None, None
    return d.get("sim_topk_hbm_bytes_per_launch"), f"profiles/pmc_{config}.json ({d.get('source', 'rocprofv3 PMC')})"


def sq_summary(config: str):
    """Executed-MFMA figures of the search's first pass from the committed SQ counter passes of THIS config
    (profiles/sq_<config>.json, tools/sq_summary.py --json), else None."""
    path = os.path.join(ROOT, "profiles", f"sq_{config}.json")
    try:
        d = json.load(open(path))
    except (OSError, ValueError):
        return None
    return d if d.get("config") == config else None


def affine_hbm_roofline(dev, K: int, n_queries: int = 262_144, reps: int = 10) -> dict:
    """k_affine on a pool larger than the 256 MB Infinity Cache, so the candidate-row gathers are HBM traffic: the cfg4
    signal (60 min, 48 kHz: 86.4 M domains, a 2.76 GB pool), the real candidates of its first `n_queries` ranges
    (searched against the whole table), the kernel timed alone with HIP events on its stream.  Cold: a 1 GiB buffer is
    rewritten before every launch (the pipeline's case: the search streams the whole fp16 table right before the
    solve); warm: back to back.  The solve's memory side is 64 random 32-B rows per range, which HBM serves at a
    request-rate limit far below its streaming peak: `gather_ceiling` measures that limit on this device
    (fwav_debug_gather_rows: the same number of uniformly random rows of the same pool, nothing computed)."""
    from fwav import engine, synth
    from fwav._lib import call
    sig_h, _, _ = synth.make_config_signal("cfg4")
    sig = torch.from_numpy(sig_h).to(dev)
    res = engine.compress_device(sig, 2048, K, shard=(0, n_queries), keep_intermediates=True)
    nd, rs, q = res.n_domains, res.range_size, n_queries
    out = [torch.empty(q, dtype=dt, device=dev) for dt in (torch.int32, torch.float32, torch.float32, torch.uint8,
                                                           torch.float32)]
    st = torch.cuda.current_stream(dev)
    args = (res.ranges.data_ptr(), q, rs, res.cand.data_ptr(), K, res.pool.data_ptr(), nd, 16.0,
            *[t.data_ptr() for t in out], st.cuda_stream)
    flush = torch.empty(1 << 28, dtype=torch.float32, device=dev)
    sink = torch.empty(1, dtype=torch.float32, device=dev)

    def timed(fn, cold):
        fn()
        ms = []
        for _ in range(reps):
            if cold:
                flush.fill_(1.0)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            fn()
            e1.record(st)
            torch.cuda.synchronize(dev)
            ms.append(e0.elapsed_time(e1))
        return sorted(ms)[len(ms) // 2]

    ms_cold = timed(lambda: call("fwav_affine", *args), True)
    ms_warm = timed(lambda: call("fwav_affine", *args), False)
    n_rows = q * K
    ms_gather = timed(lambda: call("fwav_debug_gather_rows", res.pool.data_ptr(), nd, rs, n_rows, sink.data_ptr(),
                                   st.cuda_stream), True)
    same = bool(torch.equal(out[0], res.idx[:q]))
    nbytes = q * (4 * rs + 4 * K + 4 * K * rs + 17)
    del res, sig, out, flush
    torch.cuda.empty_cache()
    gbs = nbytes / (ms_cold * 1e-3) / 1e9
    ceil_gbs = n_rows * 4 * rs / (ms_gather * 1e-3) / 1e9
    return {"bound": "hbm", "achieved": gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": gbs / HBM_PEAK_GBS,
            "bytes_per_launch": nbytes, "launch_ms": ms_cold, "cache": "cold (1 GiB rewritten before each launch)",
            "warm": {"launch_ms": ms_warm, "achieved": nbytes / (ms_warm * 1e-3) / 1e9},
            "gather_ceiling": {"rows_per_s": n_rows / (ms_gather * 1e-3), "row_bytes_gbs": ceil_gbs,
                               "note": f"{n_rows} uniformly random {4 * rs}-B rows of the same pool, cold, nothing "
                                       f"computed (fwav_debug_gather_rows)"},
            "rows_per_s": n_rows / (ms_cold * 1e-3),
            # the north star's ≥ 60 % HBM stated against what random 32-B rows allow on this chip: the solve's row rate
            # over the gather-only ceiling's (> 1: candidate rows cluster, so the L2 dedups neighbouring ranges' rows)
            "frac_of_gather_ceiling": ms_gather / ms_cold,
            "equals_pipeline_output": same,
            "workload": f"cfg4 (60 min 48 kHz noise): the real top-{K} candidates of its first {q} ranges, pool of "
                        f"{nd} rows ({nd * rs * 4 / 1e9:.2f} GB, above the 256 MB MALL)"}


def rank_share_roofline(sig, tile: int, K: int, nr: int, nd: int, world: int = 8, reps: int = 7) -> dict:
    """The search of ONE rank's share at N = `world` (the last rank's contiguous block; cfg2 noise prunes nothing, so
    the prune-balanced split of fwav.dist is the even one): its first pass + merge by HIP events on the launch
    stream, as the algorithmic rate of the full-size line."""
    from fwav import engine
    lo = nr - nr // world
    ms = []
    for i in range(reps + 2):
        ev = {}
        r = engine.compress_device(sig, tile, K, energy_thresh=1e-4, shard=(lo, nr), events=ev, defer_ties=True)
        r.wait()
        torch.cuda.synchronize()
        if i >= 2:
            ms.append(ev["sim_topk"][0].elapsed_time(ev["sim_topk"][1]))
    t = sorted(ms)[len(ms) // 2]
    q = int(r.n_active.item())
    tf = 2.0 * q * nd * 16 / (t * 1e-3) / 1e12
    return {"world": world, "queries": q, "launch_ms": t, "achieved": tf, "unit": "TFLOP/s",
            "frac": tf / F16_MFMA_PEAK_TF, "work": f"2*{q}*{nd}*16 flop (algorithmic, as `roofline`)",
            "note": "median of the sim_topk stage over the reps; one rank's compute only (no broadcast / gather)"}


def fwav_io_bench() -> dict:
    """SURVEY §8(f) rank 1 at the size that motivates it: save_compressed / load_compressed of a cfg4-shaped .fwav
    (86,398,977 x 8 domain rows + 21,600,000 match records = 3.13 GB).  Values are seeded random (the I/O path does
    not look at them; byte identity with the reference's format is tests/test_host.py's job)."""
    import tempfile
    from fwav import fwavio
    from fwav.matches import MatchList
    nd, nr, rs = 86_398_977, 21_600_000, 8
    rng = np.random.default_rng(0)
    dom = rng.standard_normal((nd, rs), dtype=np.float32)
    m = MatchList(rng.integers(0, nd, nr, dtype=np.int32), rng.standard_normal(nr, dtype=np.float32),
                  rng.standard_normal(nr, dtype=np.float32), rng.integers(0, 2, nr, dtype=np.uint8),
                  rng.random(nr, dtype=np.float32))
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "cfg4.fwav")
        t0 = time.perf_counter()
        fwavio.save_compressed(p, m, dom, rs, 48000, 4, 2048, 2, 1e-4, 172_800_000)
        t_save = time.perf_counter() - t0
        size = os.path.getsize(p)
        t0 = time.perf_counter()
        out = fwavio.load_compressed(p)
        t_load = time.perf_counter() - t0
        ok = bool(np.array_equal(out[1], dom) and np.array_equal(out[0].idx, m.idx) and np.array_equal(out[0].err, m.err))
    return {"bytes": size, "save_ms": t_save * 1e3, "save_gbs": size / t_save / 1e9, "load_ms": t_load * 1e3,
            "load_gbs": size / t_load / 1e9, "roundtrip_equal": ok, "checksum": "SHA-256 verified on load",
            "note": "cfg4 shape, seeded random values; one SHA-256 stream over the body bounds both directions"}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    # FWAV_BENCH_BACKEND=gloo + FWAV_BENCH_SHARE_GPU=1 rehearse the multi-rank path on a one-GPU box (ranks share
    # cuda:0, collectives on host tensors); the driver's N-GPU runs use the default: RCCL, one GPU per rank.
    backend = os.environ.get("FWAV_BENCH_BACKEND", "nccl")
    dev_index = local % torch.cuda.device_count() if os.environ.get("FWAV_BENCH_SHARE_GPU") else local
    torch.cuda.set_device(dev_index)
    # FWAV_BENCH_FORCE_DIST=1 runs the multi-rank path at world size 1 (its collectives included) — a check of the
    # RCCL calls on a one-GPU box; the value is then the sharded path's, not the N = 1 line
    sharded = world > 1 or bool(os.environ.get("FWAV_BENCH_FORCE_DIST"))
    if sharded:
        import torch.distributed as dist  # noqa: F811
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group(backend)
    import __graft_entry__
    __graft_entry__.build()
    from fwav import api, engine, synth
    from fwav import dist as fdist

    dev = torch.device("cuda", dev_index)
    cfg = synth.CONFIGS[args.config]
    tile, K = cfg["tile"], cfg["top_k"]
    sig_h, sr, sw = synth.make_config_signal(args.config, seconds=args.seconds, seed=0)
    sig = torch.from_numpy(sig_h).to(dev) if rank == 0 else None
    torch.cuda.synchronize()

    phase = {}
    # --streams S > 1: consecutive calls alternate over S HIP streams, so that one call's search can start on the CUs
    # the previous call's last workgroups leave idle (each call's kernels stay in order on its own stream).  Every N
    # runs the same count (the driver's 1 -> 8 curve must compare like with like; N = 1 measured 17.2
    # vs 17.8 ms per step with two streams vs one, profiles/r05/bench_streams{1,2}.log).  With overlapping launches
    # a launch's own HIP-event duration is stretched by the other stream's, so the roofline is timed on extra
    # single-stream steps after the timed region (solo_search_ms).
    n_streams = args.streams
    streams = [torch.cuda.current_stream(dev)] + [torch.cuda.Stream(dev) for _ in range(max(1, n_streams) - 1)]
    nstep = [0]

    def call_stream():
        nstep[0] += 1
        return streams[(nstep[0] - 1) % len(streams)]

    if not sharded:
        def step(ev=None):
            # the host half of numpy-order tie resolution (a few rows per step) overlaps the next step's search;
            # every step's outputs are final (wait()) before the timed region closes
            with torch.cuda.stream(call_stream()):
                r = engine.compress_device(sig, tile, K, energy_thresh=1e-4, events=ev, defer_ties=True,
                                           tie_order=args.tie_order)
            step.pending.append(r)
            return r
    else:
        LAG = 3  # started calls in flight before the oldest is finished (its ties waited for, its matches gathered)

        def step(ev=None, phases=False):
            def compute(s, t, k, thr, shard):
                r = engine.compress_device(s, t, k, energy_thresh=thr, shard=shard, events=ev, defer_ties=not phases,
                                           tie_order=args.tie_order)
                step.last = r
                step.sig_local = s
                return None if r.empty else dict(idx=r.idx, s=r.s, o=r.o, sym=r.sym, err=r.err, pool=r.pool,
                                                 silent=r.is_silent, wait=r.wait)
            # every rank knows the configuration's signal length; per-phase host timings (which synchronise the
            # device at each phase boundary) are taken on extra unpipelined steps after the timed ones
            tm = {} if phases else None
            cs = call_stream() if not phases else streams[0]
            with torch.cuda.stream(cs):
                h = fdist.compress_sharded_start(sig, tile, K, 1e-4, device=dev, compute=compute, timings=tm,
                                                 n=int(sig_h.size), signal_ready=True)
            h["stream"] = cs
            if phases:
                step.out = fdist.compress_sharded_finish(h)
                for k_, v in tm.items():
                    phase.setdefault(k_, []).append(v)
            else:
                # like N = 1's deferred ties: a call's host tie ranking overlaps the next calls' searches, and its
                # gather follows once it is final; every started call is finished inside the timed region (drain)
                step.inflight.append(h)
                while len(step.inflight) > LAG:
                    step.out = finish(step.inflight.pop(0))
            return step.last

        def finish(h):
            with torch.cuda.stream(h["stream"]):  # the gather on the call's own stream
                return fdist.compress_sharded_finish(h)

        step.inflight = []

    if not sharded:
        step.pending = []

    def drain():
        for r in getattr(step, "pending", []):
            r.wait()
        if not sharded:
            step.pending = []
        while getattr(step, "inflight", None):
            step.out = finish(step.inflight.pop(0))

    for _ in range(args.warmup):
        res = step()
    drain()
    torch.cuda.synchronize()
    phase.clear()

    def barrier():
        if dist is not None:
            dist.barrier()

    evs = []
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ev = {}
        res = step(ev)
        evs.append(ev)
    drain()
    torch.cuda.synchronize()
    barrier()
    dt = time.perf_counter() - t0
    stage_ms = {s: float(np.mean([e[s][0].elapsed_time(e[s][1]) for e in evs])) for s in STAGES if s in evs[0]}
    n_active = int(res.n_active.item())
    nr, nd, rs = res.n_ranges, res.n_domains, res.range_size
    per_rank = None
    if dist is not None:
        for _ in range(3):  # phase breakdown (untimed)
            step(phases=True)
        torch.cuda.synchronize()
        cd = dev if backend == "nccl" else torch.device("cpu")
        t = torch.tensor([dt], dtype=torch.float64, device=cd)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        mine = torch.tensor([stage_ms.get("sim_topk", 0.0), float(n_active), res.shard[1] - res.shard[0],
                             *[float(np.mean(phase.get(k_, [0.0]))) * 1e3 for k_ in ("broadcast_s", "compute_s",
                                                                                      "gather_s")]],
                            dtype=torch.float64, device=cd)
        allr = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allr, mine)
        per_rank = [dict(zip(("sim_topk_ms", "active_queries", "ranges", "broadcast_ms", "compute_ms", "gather_ms"),
                             [float(x) for x in a.cpu().tolist()])) for a in allr]
    ms = dt / args.steps * 1e3
    value = nr / (dt / args.steps)

    # the roofline's launch time: with several streams the timed launches overlap (each one's HIP-event span includes
    # the other stream's work), so the search is re-timed alone, on one stream, over untimed extra calls of the same
    # shard (its kernels and outputs are those of the timed calls)
    solo_ms = None
    if len(streams) > 1:
        s_loc = sig if not sharded else getattr(step, "sig_local", None)
        if s_loc is not None:
            solo = []
            for i in range(6):
                ev = {}
                r_ = engine.compress_device(s_loc, tile, K, energy_thresh=1e-4, shard=res.shard if sharded else None,
                                            events=ev, defer_ties=True)
                r_.wait()
                torch.cuda.synchronize()
                if i:
                    solo.append(ev["sim_topk"][0].elapsed_time(ev["sim_topk"][1]))
            solo_ms = float(sorted(solo)[len(solo) // 2])
    t_topk = (solo_ms if solo_ms is not None else stage_ms["sim_topk"]) * 1e-3
    flops = 2.0 * n_active * nd * 16
    achieved_tf = flops / t_topk / 1e12
    traffic, traffic_src = pmc_traffic(args.config) if not sharded else (None, None)
    line = {
        "metric": "ranges matched/sec at tile_size=2048, top-K=64",
        "value": value, "unit": "ranges/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": ms, "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": "f32", "data": f"synthetic ({args.config} generator, seed 0; one signal, ranges sharded over ranks)"
                                + ("" if args.tie_order == "numpy" else f"; tie_order={args.tie_order} (diagnostic)"),
        "config": {"workload": f"{args.config}: {sig_h.size / sr:.0f} s {sr} Hz "
                               f"{WORKLOAD_TEXT.get(args.config, '').split(' ', 4)[-1]}, tile_size={tile}, "
                               f"top_k={K}, n_ranges={nr}, n_domains={nd}",
                   "tile_size": tile, "top_k": K, "n_ranges": nr, "n_domains": nd,
                   "parallelism": "single GPU" if not sharded else f"ranges sharded x{world} (RCCL broadcast + "
                                                                  f"gather)",
                   "streams": len(streams)},
        "roofline": {"kernel": f"{TOPK_KERNEL} (fp16 MFMA similarity GEMM pre-filter + streaming exact top-K)",
                     "bound": "mfma", "achieved": achieved_tf, "peak": F16_MFMA_PEAK_TF, "unit": "TFLOP/s",
                     "frac": achieved_tf / F16_MFMA_PEAK_TF, "traffic": traffic, "traffic_source": traffic_src,
                     "work_per_launch": f"2*{n_active}*{nd}*16 = {flops:.4g} flop: the ALGORITHMIC work of the "
                                        f"reference's scores (every query-domain pair, fractal.py:537). The kernel "
                                        f"does not execute it all: a centroid bound skips the (tile, query set) pairs "
                                        f"that cannot reach a member's band, so `frac` is an effective rate; the "
                                        f"MFMA work actually executed is `mfma_executed`",
                     "launch_ms": t_topk * 1e3, "rank": rank,
                     **({"launch_ms_overlapped": stage_ms["sim_topk"],
                         "note": f"{len(streams)} streams in the timed steps: their launches overlap, so launch_ms is "
                                 "the same search timed alone on one stream (median of 5 extra calls); "
                                 "launch_ms_overlapped is the timed launches' own span"} if solo_ms is not None else {})},
        "stage_ms": stage_ms,
    }
    sq = sq_summary(args.config) if not sharded else None
    if sq and sq.get("mfma_executed_flop_per_launch"):
        ex_tf = sq["mfma_executed_flop_per_launch"] / t_topk / 1e12
        line["roofline"]["mfma_executed"] = {
            "flop_per_launch": sq["mfma_executed_flop_per_launch"], "achieved": ex_tf, "unit": "TFLOP/s",
            "frac": ex_tf / F16_MFMA_PEAK_TF, "mfma_busy": sq.get("mfma_busy_frac"),
            "wave_time": sq.get("wave_time"),
            "note": "SQ_INSTS_MFMA x 32,768 flop (v_mfma_f32_32x32x16_f16) from the committed SQ pass of this config, "
                    "over this run's launch time; mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / SIMD cycles",
            "source": f"profiles/sq_{args.config}.json ({sq.get('source')})"}
    if traffic:
        # the north star's "fraction of the HBM roofline" for the same launch: measured HBM bytes (PMC) over its time
        # (the kernel is bound by MFMA/VALU issue, not by HBM: its table is re-read from the Infinity Cache)
        hbm = traffic / t_topk / 1e9
        line["roofline"]["hbm"] = {"achieved": hbm, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": hbm / HBM_PEAK_GBS}
    if per_rank is not None:
        line["per_rank"] = per_rank
    extras = not sharded and not args.no_extras
    if extras:
        # Host-boundary rate (not `value`): numpy signal in host memory → matches (SoA) back in host memory.
        def e2e_step():
            r = engine.compress_device(torch.from_numpy(sig_h).to(dev), tile, K, energy_thresh=1e-4)
            return [t.cpu() for t in (r.idx, r.s, r.o, r.sym, r.err)]

        e2e_step()
        torch.cuda.synchronize()
        n_e = max(1, min(args.steps, 3))
        te0 = time.perf_counter()
        for _ in range(n_e):
            e2e_step()
        e2e_ms = (time.perf_counter() - te0) / n_e * 1e3
        api.compress_audio(sig_h, sr, 4, tile_size=tile, top_k=K, device=dev)
        torch.cuda.synchronize()
        ta0 = time.perf_counter()
        for _ in range(n_e):
            out_api = api.compress_audio(sig_h, sr, 4, tile_size=tile, top_k=K, device=dev)
        api_ms = (time.perf_counter() - ta0) / n_e * 1e3
        assert len(out_api[0]) == out_api[2]
        line["host_boundary"] = {"ms_per_step": e2e_ms, "ranges_per_s": nr / (e2e_ms * 1e-3),
                                 "note": "host numpy signal in -> host SoA matches out (PCIe both ways); not `value`"}
        line["api_call"] = {"ms_per_call": api_ms, "ranges_per_s": nr / (api_ms * 1e-3),
                            "note": "fractal.compress_audio(): host signal in, MatchList + domain pool out"}

        # Decode (the metric's second half, "reconstruction SNR dB"): reference defaults (8 iterations, eps 1e-3)
        # and a forced 50-iteration run (eps 0, the cfg5 protocol at this config's size).
        dec = {}
        for name, iters, eps in (("default", 8, 1e-3), ("forced50", 50, 0.0)):
            engine.decompress_device(res.idx, res.s, res.o, res.sym, res.pool, nr, rs, iters, eps)
            torch.cuda.synchronize()
            reps = 5
            td0 = time.perf_counter()
            for _ in range(reps):
                rec, ran, _ = engine.decompress_device(res.idx, res.s, res.o, res.sym, res.pool, nr, rs, iters, eps)
            torch.cuda.synchronize()
            tdec = (time.perf_counter() - td0) / reps
            snr = api.compute_snr(sig_h, rec[:sig_h.size].cpu().numpy())
            dec[name] = {"iterations": ran, "ms": tdec * 1e3, "snr_db": snr,
                         "range_iterations_per_s": nr * ran / tdec}
        dec["note"] = ("iteration-resident kernel: up to 64 iterations per launch with each range's reconstruction "
                       "in registers; per-iteration streaming would move (12*rs+17) B/range/iteration = "
                       f"{nr * (12 * rs + 17) / 1e6:.1f} MB per iteration")
        dec["streaming_equivalent_gbs_forced50"] = nr * (12 * rs + 17) * 50 / (dec["forced50"]["ms"] * 1e-3) / 1e9
        line["decode"] = dec
        # numpy-order ties, synchronously (the timed steps defer the host half): how many rows the search lists, how
        # many the device-side check sends to numpy, and what that costs in one call
        tev = {}
        rt = engine.compress_device(sig, tile, K, energy_thresh=1e-4, events=tev)
        torch.cuda.synchronize()
        line["ties"] = {"rows_with_exact_ties": rt.n_ties, "rows_ranked_by_numpy": rt.n_resolved,
                        "ms_synchronous": tev["ties"][0].elapsed_time(tev["ties"][1]),
                        "note": "timed steps overlap this host work with the next step's search (defer_ties)"}
        try:
            line["fwav_io_cfg4"] = fwav_io_bench()
        except Exception as e:  # noqa: BLE001
            line["fwav_io_cfg4"] = {"error": str(e)[:200]}
        line["roofline_rank_share"] = rank_share_roofline(sig, tile, K, nr, nd)
        line["roofline_affine"] = affine_hbm_roofline(dev, K)
        line["roofline_affine_in_pipeline"] = {
            "achieved": nr * (4 * rs + 4 * K + 4 * K * rs + 17) / (stage_ms["affine"] * 1e-3) / 1e9,
            "unit": "GB/s", "note": f"{args.config}'s own pool ({nd * rs * 4 / 1e6:.0f} MB) is served from MALL"}
        if rank == 0 and not args.no_cpu_baseline:
            try:
                cmd = [sys.executable, os.path.join(ROOT, "oracle", "cpu_baseline.py"), "--config", args.config]
                if args.cpu_workers:
                    cmd += ["--workers", str(args.cpu_workers)]
                out = subprocess.run(cmd, capture_output=True, text=True, timeout=400)
                cpu = json.loads(out.stdout.strip().splitlines()[-1])
            except Exception as e:  # noqa: BLE001
                cpu = {"error": str(e)[:200]}
            line["cpu_baseline"] = cpu
            if cpu and "value" in cpu:
                line["gpu_over_cpu"] = value / cpu["value"]
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
