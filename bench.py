#!/usr/bin/env python3
"""Benchmark: ranges matched/sec at tile_size=2048, top-K=64 (BASELINE.json metric) on MI355X.

One step = one full compress hot path over one 60 s 44.1 kHz noise signal (cfg2, BASELINE.json configs[1]):
voiced detection → ranges → domain pool → embeddings → energy prune → similarity top-64 → affine solve with
mirror, all on device; the signal is resident in HBM before the timed region and the match arrays stay there.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N): every rank compresses its
own cfg2 signal (independent objects, seed = rank; no collective on the data path) → "scaling": "weak";
value = N · n_ranges / max-over-ranks time.  The single-file range-sharded path (RCCL broadcast of the
signal + gather of matches) is fwav.dist and is exercised by tests, not by this line.

Also reported: the dominant kernel's roofline (similarity top-K, fp32 MFMA bound; HIP events on the stream
the kernels are launched on), the affine solver's HBM roofline (the north star's ≥60 % target), per-stage
times, and the CPU baseline (oracle restatement on this host, bounded sample, rank 0 at N=1 only).
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
FP32_MFMA_PEAK_TF = 157.3    # dense f32 MFMA (= f32 vector) peak
F16_MFMA_PEAK_TF = 2516.6    # dense f16 MFMA peak: v_mfma_f32_32x32x16_f16, 32 cycles/SIMD, 1024 SIMDs, 2.4 GHz
STAGES = ["voiced_ranges", "pool_embed", "prune", "sim_topk", "affine"]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--seconds", type=float, default=None, help="override signal length (debug)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-workers", type=int, default=8)
    return ap.parse_args()


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
    if world > 1:
        import torch.distributed as dist  # noqa: F811
        torch.cuda.set_device(dev_index)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group(backend)
    import __graft_entry__
    __graft_entry__.build()
    from fwav import api, engine, synth

    dev = torch.device("cuda", dev_index)
    cfg = synth.CONFIGS[args.config]
    sig_h, sr, sw = synth.make_config_signal(args.config, seconds=args.seconds, seed=rank)
    tile, K = cfg["tile"], cfg["top_k"]
    sig = torch.from_numpy(sig_h).to(dev)
    torch.cuda.synchronize()

    def step(ev=None):
        return engine.compress_device(sig, tile, K, energy_thresh=1e-4, events=ev)

    for _ in range(args.warmup):
        res = step()
    torch.cuda.synchronize()

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
    torch.cuda.synchronize()
    barrier()
    t1 = time.perf_counter()
    dt = t1 - t0
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64, device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())

    # Host-boundary rate (not `value`): numpy signal in host memory → matches (SoA) back in host memory, i.e.
    # the compress_audio boundary including PCIe both ways (DESIGN.md "Measurement").
    def e2e_step():
        r = engine.compress_device(torch.from_numpy(sig_h).to(dev), tile, K, energy_thresh=1e-4)
        return [t.cpu() for t in (r.idx, r.s, r.o, r.sym, r.err)]

    e2e_step()
    torch.cuda.synchronize()
    te0 = time.perf_counter()
    for _ in range(max(1, min(args.steps, 3))):
        e2e_step()
    e2e_ms = (time.perf_counter() - te0) / max(1, min(args.steps, 3)) * 1e3

    # The reference's own boundary: fractal.compress_audio(numpy signal) -> (MatchList, domains ndarray, ...), i.e.
    # host signal in, matches + domain pool (nd x rs f32) on the host.
    sr_api = synth.CONFIGS[args.config]["sr"]
    api.compress_audio(sig_h, sr_api, 4, tile_size=tile, top_k=K, device=dev)
    torch.cuda.synchronize()
    ta0 = time.perf_counter()
    n_api = max(1, min(args.steps, 3))
    for _ in range(n_api):
        out_api = api.compress_audio(sig_h, sr_api, 4, tile_size=tile, top_k=K, device=dev)
    api_ms = (time.perf_counter() - ta0) / n_api * 1e3
    assert len(out_api[0]) == out_api[2]

    # Decode (the metric's second half, "reconstruction SNR dB"): the reference defaults (8 iterations,
    # eps 1e-3) and a forced 50-iteration run (eps 0, SURVEY §8(d) cfg5 protocol at this config's size).
    dec = {}
    for name, iters, eps in (("default", 8, 1e-3), ("forced50", 50, 0.0)):
        engine.decompress_device(res.idx, res.s, res.o, res.sym, res.pool, res.n_ranges, res.range_size, iters, eps)
        torch.cuda.synchronize()
        td0 = time.perf_counter()
        rec, ran, _ = engine.decompress_device(res.idx, res.s, res.o, res.sym, res.pool, res.n_ranges,
                                               res.range_size, iters, eps)
        torch.cuda.synchronize()
        tdec = time.perf_counter() - td0
        snr = api.compute_snr(sig_h, rec[:sig_h.size].cpu().numpy())
        dec[name] = {"iterations": ran, "ms": tdec * 1e3, "snr_db": snr}
    nr_, rs_ = res.n_ranges, res.range_size
    dec["bytes_per_iteration"] = nr_ * (12 * rs_ + 17)  # fwav_decode.hip header
    dec["iteration_gbs"] = dec["bytes_per_iteration"] / (dec["forced50"]["ms"] * 1e-3 / 50) / 1e9

    nr, nd, rs = res.n_ranges, res.n_domains, res.range_size
    n_active = int(res.n_active.item())
    stage_ms = {s: float(np.mean([e[s][0].elapsed_time(e[s][1]) for e in evs])) for s in STAGES}
    t_topk = stage_ms["sim_topk"] * 1e-3
    t_aff = stage_ms["affine"] * 1e-3
    flops = 2.0 * n_active * nd * 16
    aff_bytes = nr * (4 * rs + 4 * K + 4 * K * rs + 17)
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_latest.json")
    if os.path.exists(pmc):
        try:
            traffic = json.load(open(pmc)).get("sim_topk_hbm_bytes_per_launch")
        except Exception:  # noqa: BLE001
            traffic = None
    achieved_tf = flops / t_topk / 1e12
    aff_gbs = aff_bytes / t_aff / 1e9
    ms = dt / args.steps * 1e3
    value = world * nr / (dt / args.steps)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            out = subprocess.run([sys.executable, os.path.join(ROOT, "oracle", "cpu_baseline.py"), "--config",
                                  args.config, "--workers", str(args.cpu_workers)], capture_output=True, text=True,
                                 timeout=300)
            cpu = json.loads(out.stdout.strip().splitlines()[-1])
        except Exception as e:  # noqa: BLE001
            cpu = {"error": str(e)[:200]}
    if rank == 0:
        line = {
            "metric": "ranges matched/sec at tile_size=2048, top-K=64",
            "value": value, "unit": "ranges/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f32", "data": "synthetic (seeded clip(N(0,0.25^2)) noise, one signal per rank)",
            "config": {"workload": f"{args.config}: {sig_h.size / sr:.0f} s {sr} Hz mono noise, tile_size={tile}, "
                                   f"top_k={K}, n_ranges={nr}, n_domains={nd}", "tile_size": tile, "top_k": K,
                       "n_ranges": nr, "n_domains": nd, "active_queries": n_active, "parallelism": f"replicas{world}"},
            "roofline": {"kernel": "k_sim_topk_f16 (fp16 MFMA similarity GEMM pre-filter + streaming exact top-K)",
                         "bound": "mfma", "achieved": achieved_tf, "peak": F16_MFMA_PEAK_TF, "unit": "TFLOP/s",
                         "frac": achieved_tf / F16_MFMA_PEAK_TF, "traffic": traffic,
                         "work_per_launch": f"2*{n_active}*{nd}*16 = {flops:.4g} flop (one fp16 MFMA score per "
                                            f"query-domain pair; exact f32 rescoring of survivors not counted)",
                         "launch_ms": t_topk * 1e3},
            "roofline_affine": {"bound": "hbm", "achieved": aff_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": aff_gbs / HBM_PEAK_GBS, "bytes_per_launch": aff_bytes},
            "stage_ms": stage_ms,
            "host_boundary": {"ms_per_step": e2e_ms, "ranges_per_s": world * nr / (e2e_ms * 1e-3),
                              "note": "host numpy signal in -> host SoA matches out (PCIe both ways); not `value`"},
            "api_call": {"ms_per_call": api_ms, "ranges_per_s": world * nr / (api_ms * 1e-3),
                         "note": "fractal.compress_audio(): host signal in, MatchList + domain pool out; not `value`"},
            "decode": dec,
            "cpu_baseline": cpu,
        }
        if cpu and "value" in cpu:
            line["gpu_over_cpu"] = value / cpu["value"]
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
