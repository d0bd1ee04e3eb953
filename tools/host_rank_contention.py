"""Host cost of numpy's tie ranking at cfg4 row width with several ranks ranking at once.

The exact tie order of the reference (fractal.py:537-541: argpartition of the whole 86.4 M-score row, then argsort
of the K) is numpy's; fwav.ties ranks each listed row on the host with numpy's own calls.  At 8 ranks on one node,
eight processes rank their rows at the same time through one host memory system.  This measures, on the box it runs
on: the time of one 86.4 M-float row ranked by `fwav.nporder.numpy_topk_row` with P concurrent processes, each with
T ranking threads (the product's pool: FWAV_TIE_THREADS, default 8), and projects one rank's eighth of cfg4 (151
ranked rows per call, profiles/r03/sub_blocks_cfg4_eighth.log) against its 7.3 s search.

Rows: synthetic f32 scores shaped like cfg4's (values near 1.9 with a long lower tail, many exact duplicates at the
top — the rows numpy must order); argpartition's cost is dominated by the row's size (memory traffic of the scores
and its 8-byte index array), not by the values.
usage: python tools/host_rank_contention.py [--rows R] [--procs 1,2,4,8] [--threads 1,2,8]
"""
import argparse
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "audio-compression_amd")]

ND = 86_398_977  # cfg4's domains
K = 64


def _row(seed: int):
    import numpy as np
    rng = np.random.default_rng(seed)
    x = (1.95 - np.abs(rng.standard_normal(ND, dtype=np.float32)) * np.float32(0.35)).astype(np.float32)
    x[rng.integers(0, ND, 4096)] = np.float32(1.9990234)  # a block of exact ties at the top
    return x


def _worker(args):
    pid, rows, threads, start_evt, q = args
    from concurrent.futures import ThreadPoolExecutor

    from fwav.nporder import numpy_topk_row
    data = [_row(1000 * pid + i) for i in range(min(rows, 2))]
    start_evt.wait()
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        futs = [ex.submit(numpy_topk_row, data[i % len(data)], K) for i in range(rows)]
        for f in futs:
            f.result()
    q.put((pid, time.perf_counter() - t0))


def run(procs: int, threads: int, rows: int) -> float:
    ctx = mp.get_context("spawn")
    evt = ctx.Manager().Event()
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=((p, rows, threads, evt, q),)) for p in range(procs)]
    for p in ps:
        p.start()
    time.sleep(2.0 + 0.5 * procs)  # every process has built its rows
    evt.set()
    out = [q.get(timeout=900) for _ in ps]
    for p in ps:
        p.join()
    return max(t for _, t in out) / rows  # seconds per row in the slowest process


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=8)
    ap.add_argument("--procs", default="1,8")
    ap.add_argument("--threads", default="1,2,8")
    a = ap.parse_args()
    try:
        share = len(os.sched_getaffinity(0))
    except AttributeError:
        share = os.cpu_count()
    print(f"host: os.cpu_count()={os.cpu_count()}, affinity {share} CPUs, OMP_NUM_THREADS="
          f"{os.environ.get('OMP_NUM_THREADS')}; row = {ND} f32 ({ND * 4 / 1e6:.0f} MB) + its int64 index "
          f"array ({ND * 8 / 1e6:.0f} MB)", flush=True)
    base = None
    for P in [int(x) for x in a.procs.split(",")]:
        for T in [int(x) for x in a.threads.split(",")]:
            spr = run(P, T, a.rows)
            if base is None:
                base = spr
            eighth = 151 * spr
            print(f"procs {P} x threads {T}: {spr * 1e3:7.1f} ms per row in the slowest process "
                  f"({base / spr:4.2f}x the first line's rate per process); one rank's eighth of cfg4 (151 rows): "
                  f"{eighth:5.2f} s of host ranking vs its 7.3 s search", flush=True)


if __name__ == "__main__":
    main()
