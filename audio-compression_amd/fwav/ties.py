"""Exactly tied similarity scores: the reference's numpy tie order, reproduced where it can change a match.

The reference ranks each range's candidates with numpy (fractal.py:535-541)::

    scores = domain_embs @ q
    idxs = np.argpartition(scores, -top_k)[-top_k:]
    return idxs[np.argsort(scores[idxs])[::-1]]

so among exactly equal scores its order — and, when the K-th and (K+1)-th scores are equal, its candidate set — is
whatever numpy's selection and sort (x86-simd-sort on this image's CPUs) leave them in: a function of the whole
score row, not of the tied values alone.  The device search emits (score desc, index asc) and lists every query
whose top K + 1 scores hold a tie (``fwav_sim_topk`` ``ties``); ``fwav_tie_check`` keeps those whose match could
depend on the order (a tie at the K-th place, or two candidates of one run of equal scores that both attain the
minimum error).  For them — none on noise, a handful of rows on speech, many on periodic signals — this module
takes the exact score row (``fwav_score_rows``, the reference's own sgemv order), runs the reference's own numpy
calls on it (:func:`numpy_topk_row`), and re-solves those rows with ``fwav_affine``.  Every value still comes from
the device; numpy only orders equal keys, exactly as it does in the reference.
"""
from __future__ import annotations

import os
import threading
import time

import numpy as np
import torch

from ._lib import call
from .nporder import blas_threads, numpy_topk_row  # noqa: F401  (re-exported: the numpy-only half of this module)

#: device bytes of exact score rows computed per fwav_score_rows launch (the launch reads the embedding table once)
DEVICE_ROW_BUDGET = 2 << 30
#: page-locked host bytes of score rows in flight (one slot per row being ranked)
HOST_ROW_BUDGET = 4 << 30
MAX_SLOTS = 64
#: device bytes of score rows queued at once between the query sub-blocks of a search (fwav.engine): all of a
#: sub-block's rows in one launch, so that none waits behind the next sub-block's search
PIPE_ROW_BUDGET = 16 << 30

_TRACE = bool(os.environ.get("FWAV_TIES_TRACE"))


_POOL = None
_SLOTS: list = []
_SLOT_BUSY: list = []  # per staging slot: the future ranking the row it holds (None when free)
_SLOT_LOCK = threading.Lock()  # one staging loop at a time owns the slot ring
_SLOT_NEXT = 0
_DRIVER = None
_SIDE: dict = {}
_COPY: dict = {}


def _driver():
    global _DRIVER
    if _DRIVER is None:
        from concurrent.futures import ThreadPoolExecutor
        _DRIVER = ThreadPoolExecutor(1, thread_name_prefix="fwav-ties-driver")
    return _DRIVER


def defer(finish, device: torch.device):
    """Run ``finish(stream)`` — the host half of a tie resolution — on the background driver thread, on a side stream
    that first waits for everything queued so far on ``device``'s current stream.  Returns the Future of its result.
    One driver thread: resolutions run in call order."""
    ev = torch.cuda.Event()
    ev.record(torch.cuda.current_stream(device))
    key = str(device)
    if key not in _SIDE:
        # (a high-priority stream was measured no better: its kernels still wait behind the next call's search,
        # which holds every CU — profiles/r03/ties_defer_cfg3.log)
        _SIDE[key] = torch.cuda.Stream(device)
    side = _SIDE[key]

    def job():
        with torch.cuda.device(device), torch.cuda.stream(side):
            side.wait_event(ev)
            out = finish(side.cuda_stream)
            side.synchronize()
            return out

    return _driver().submit(job)


def _cpu_share() -> int:
    """CPUs this process may use: the cgroup's CPU quota (cpu.max) when it sets one, else the affinity mask (the GPU
    boxes report 256 CPUs to os.cpu_count() but give a job a 16-CPU quota)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(quota) // int(period)))
    except (OSError, ValueError):
        pass
    return max(1, n)


def tie_threads() -> int:
    """Host threads ranking exact score rows in this process: FWAV_TIE_THREADS, else the CPU share divided among the
    node's ranks (LOCAL_WORLD_SIZE), at most 8.  Measured on a GPU box with cfg4 rows (86.4 M scores,
    tools/host_rank_contention.py, profiles/r04/host_rank_contention.log): one process 8 threads 47 ms per row; eight
    processes at once 8 threads each 354 ms, 2 threads each 166 ms, 1 thread each 283 ms."""
    env = os.environ.get("FWAV_TIE_THREADS")
    if env:
        return max(1, int(env))
    ranks = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1")))
    return max(1, min(8, _cpu_share() // ranks))


def _pool():
    """Host threads for numpy's ranking of the exact score rows (argpartition runs outside the GIL): tie_threads()."""
    global _POOL
    if _POOL is None:
        from concurrent.futures import ThreadPoolExecutor
        _POOL = ThreadPoolExecutor(tie_threads(), thread_name_prefix="fwav-ties")
    return _POOL


def _slot(i: int, numel: int) -> torch.Tensor:
    """Reusable page-locked staging row i (float32), grown on demand (caller holds _SLOT_LOCK, slot i free)."""
    while len(_SLOTS) <= i:
        _SLOTS.append(None)
    t = _SLOTS[i]
    if t is None or t.numel() < numel:
        t = torch.empty(numel, dtype=torch.float32, pin_memory=True)
        _SLOTS[i] = t
    return t[:numel]


def score_row_launches(rows: torch.Tensor, *, emb: torch.Tensor, n_domains: int, q_offset: int, threads: int,
                       stream: int, budget: int = DEVICE_ROW_BUDGET, first_row: int = 0):
    """Yield (first row + first_row, device f32[m·nd] scores, event) per fwav_score_rows launch of at most
    ``budget`` bytes, each launch queued on the current stream (``stream``) when the generator reaches it.  A
    consumer that must hold one launch at a time delegates with ``yield from`` (a loop variable of its own would keep
    the previous launch alive while this generator allocates the next)."""
    nd = int(n_domains)
    n = rows.numel()
    per = max(1, min(n, budget // (4 * nd)))
    for b0 in range(0, n, per):
        rb = rows[b0:b0 + per].contiguous()
        m = rb.numel()
        S = torch.empty(m * nd, dtype=torch.float32, device=rows.device)
        call("fwav_score_rows", emb.data_ptr(), nd, rb.data_ptr(), m, int(q_offset), int(threads), S.data_ptr(),
             stream)
        ev = torch.cuda.Event()
        ev.record()
        yield b0 + first_row, S, ev
        del S, ev  # not held while the next launch allocates: one launch's rows on the device at a time


def rank_rows(launches, n: int, n_domains: int, k: int, copy_stream=None) -> list:
    """Copy the score rows of ``launches`` (score_row_launches) to the ring of page-locked slots (HOST_ROW_BUDGET)
    in runs of at most one slot per row, one synchronisation per run, and hand each landed row to numpy's ranking on
    the host pool.  Returns the n futures (candidate rows, int32[k]).  ``copy_stream``: the copies' stream (it waits
    for each launch's event), else the current stream."""
    nd = int(n_domains)
    nslots = max(2, min(MAX_SLOTS, HOST_ROW_BUDGET // (4 * nd)))  # the ring (slots are allocated on first use)
    ex = _pool()
    futs = [None] * n
    done = torch.cuda.Event()
    global _SLOT_NEXT
    with _SLOT_LOCK:
        while len(_SLOT_BUSY) < nslots:
            _SLOT_BUSY.append(None)
        base = _SLOT_NEXT  # consecutive calls take the ring's next slots, not the ones the last call is still ranking
        for b0, S, ev in launches:
            m = S.numel() // nd
            if copy_stream is not None:
                copy_stream.wait_event(ev)
            for r0 in range(0, m, nslots):
                hs = []
                for i in range(b0 + r0, b0 + min(m, r0 + nslots)):
                    sl = (base + i) % nslots
                    if _SLOT_BUSY[sl] is not None:  # its previous row is still being ranked
                        _SLOT_BUSY[sl].result()
                        _SLOT_BUSY[sl] = None
                    h = _slot(sl, nd)
                    src = S[(i - b0) * nd:(i - b0 + 1) * nd]
                    if copy_stream is not None:
                        with torch.cuda.stream(copy_stream):
                            h.copy_(src, non_blocking=True)
                    else:
                        h.copy_(src, non_blocking=True)
                    hs.append((i, sl, h))
                if copy_stream is not None:
                    done.record(copy_stream)
                else:
                    done.record()
                done.synchronize()
                if _TRACE:
                    print(f"fwav.ties {time.perf_counter():.4f}: rows {hs[0][0]}..{hs[-1][0]} of {n} on the host",
                          flush=True)
                for i, sl, h in hs:
                    futs[i] = _SLOT_BUSY[sl] = ex.submit(numpy_topk_row, h.numpy(), k)
            src = None  # (a view of S: would keep the launch's rows allocated while the next launch allocates)
            del S
        _SLOT_NEXT = (base + n) % nslots
    return futs


#: device bytes of score rows launched eagerly (on the caller's stream, right after a slice's tie check) by all the
#: rank_rows_async calls still in flight together; a call past it launches every batch on the driver's side
PIPE_EAGER_TOTAL = 32 << 30
_EAGER_LOCK = threading.Lock()
_EAGER_BYTES = 0
_ROWS: dict = {}


def rank_rows_async(rows: torch.Tensor, *, emb: torch.Tensor, n_domains: int, q_offset: int, k: int, threads: int,
                    stream: int, budget: int = PIPE_ROW_BUDGET):
    """Queue the exact score rows of ``rows`` now — at most ``budget`` bytes of them, in one launch — and copy + rank
    them on the driver thread (copies on a copy stream that waits for the launches).  Returns a Future of the n row
    futures.  Used between the query sub-blocks of one search (fwav.engine), so that the next sub-block's search does
    not delay the score rows: only their copies and numpy's ranking overlap it.  Rows beyond the budget (a periodic
    input can tie thousands of rows, 345 MB each at cfg4) are launched by the driver thread, one budget at a time as
    the earlier ones reach the host, on a side stream that waits only for this call's point in the caller's stream
    (not for what the caller queues after it: the next slice's search).  The eager first launch is skipped when the
    calls in flight already hold PIPE_EAGER_TOTAL of eager rows, so at most max(budget, PIPE_EAGER_TOTAL) + budget
    bytes of score rows are on the device however many slices are pending."""
    global _EAGER_BYTES
    n = rows.numel()
    dev = rows.device
    cur = torch.cuda.current_stream(dev)  # the caller's stream (``stream``): the eager launch goes here
    ready = torch.cuda.Event()
    ready.record(cur)  # everything this call's rows depend on (the slice's search and tie check)
    key = str(dev)
    if key not in _COPY:
        _COPY[key] = torch.cuda.Stream(dev)
        _ROWS[key] = torch.cuda.Stream(dev)
    cs, side = _COPY[key], _ROWS[key]
    nd = int(n_domains)
    per = max(1, min(n, budget // (4 * nd))) if n else 0
    nbytes = 4 * nd * per
    with _EAGER_LOCK:
        eager = n > 0 and _EAGER_BYTES + nbytes <= max(PIPE_EAGER_TOTAL, nbytes)
        if eager:
            _EAGER_BYTES += nbytes
    first = [next(score_row_launches(rows[:per], emb=emb, n_domains=nd, q_offset=q_offset, threads=threads,
                                     stream=stream, budget=budget))] if eager else []
    rest = rows[per:] if eager else rows

    def job():
        def it():  # each launch's scores are released once its rows are on the host
            global _EAGER_BYTES
            if first:
                yield first.pop(0)
                with _EAGER_LOCK:
                    _EAGER_BYTES -= nbytes
            if rest.numel():
                with torch.cuda.stream(side):
                    side.wait_event(ready)
                    yield from score_row_launches(rest, emb=emb, n_domains=nd, q_offset=q_offset, threads=threads,
                                                  stream=side.cuda_stream, budget=budget,
                                                  first_row=per if eager else 0)
        with torch.cuda.device(dev):
            return rank_rows(it(), n, n_domains, k, copy_stream=cs)

    return _driver().submit(job)


def apply_rows(rows: torch.Tensor, futs: list, *, ranges: torch.Tensor, range_size: int, pool: torch.Tensor,
               n_domains: int, k: int, s_clip: float, cand: torch.Tensor, outs: tuple, stream: int) -> None:
    """Write numpy's candidate rows (the futures of rank_rows) into ``cand`` and re-run the affine solve for those
    rows into ``outs`` = (idx, s, o, sym, err), on the current stream (``stream``)."""
    dev = rows.device
    n = rows.numel()
    # through page-locked memory, asynchronously: a copy from pageable memory would first wait for everything queued
    # on the stream (in a stream of calls, the calls still in flight)
    newc = torch.from_numpy(np.stack([f.result() for f in futs])).pin_memory().to(dev, non_blocking=True)
    rows = rows.contiguous()
    rs = int(range_size)
    rsub = torch.empty(n * rs, dtype=torch.float32, device=dev)
    # three launches: candidate rows scattered + their ranges gathered, the affine re-solve, the outputs scattered
    call("fwav_tie_rows_in", rows.data_ptr(), n, newc.data_ptr(), k, cand.data_ptr(), ranges.data_ptr(), rs,
         rsub.data_ptr(), stream)
    tmp = [torch.empty(n, dtype=t.dtype, device=dev) for t in outs]
    call("fwav_affine", rsub.data_ptr(), n, rs, newc.data_ptr(), k, pool.data_ptr(), int(n_domains), float(s_clip),
         *[t.data_ptr() for t in tmp], stream)
    call("fwav_tie_rows_out", rows.data_ptr(), n, *[t.data_ptr() for t in tmp], *[t.data_ptr() for t in outs], stream)


def resolve_rows(rows: torch.Tensor, *, emb: torch.Tensor, n_domains: int, q_offset: int, k: int, threads: int,
                 ranges: torch.Tensor, range_size: int, pool: torch.Tensor, s_clip: float, cand: torch.Tensor,
                 outs: tuple, stream: int) -> None:
    """Rows (local indices, device int32) whose match depends on numpy's tie order: exact score rows in launches of up
    to DEVICE_ROW_BUDGET (fwav_score_rows reads the embedding table once per launch), copied to a ring of page-locked
    row slots (HOST_ROW_BUDGET), numpy's ranking of each row on a host thread pool as soon as it lands, the new
    candidate rows written back to ``cand`` and the affine solve re-run for those rows into ``outs`` =
    (idx, s, o, sym, err).  (cfg4-sized rows, 86.4 M scores: 22 rows 3.5 → 1.1 s against one 256 MB
    double buffer.)"""
    n = rows.numel()
    if n == 0:
        return
    trace = os.environ.get("FWAV_TIES_TRACE")
    t0 = time.perf_counter()
    futs = rank_rows(score_row_launches(rows, emb=emb, n_domains=n_domains, q_offset=q_offset, threads=threads,
                                        stream=stream), n, n_domains, k)
    t1 = time.perf_counter()
    for f in futs:
        f.result()
    if trace:
        print(f"fwav.ties: {n} rows x {n_domains}: {(time.perf_counter() - t0) * 1e3:.1f} ms (device score rows + "
              f"copies {(t1 - t0) * 1e3:.1f} ms, numpy tail {(time.perf_counter() - t1) * 1e3:.1f} ms)", flush=True)
    apply_rows(rows, futs, ranges=ranges, range_size=range_size, pool=pool, n_domains=n_domains, k=k, s_clip=s_clip,
               cand=cand, outs=outs, stream=stream)
