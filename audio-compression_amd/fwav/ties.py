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
import time

import numpy as np
import torch

from ._lib import call

#: device bytes of exact score rows computed per fwav_score_rows launch (the launch reads the embedding table once)
DEVICE_ROW_BUDGET = 2 << 30
#: page-locked host bytes of score rows in flight (one slot per row being ranked)
HOST_ROW_BUDGET = 4 << 30

_BLAS_THREADS = None


def blas_threads() -> int:
    """OpenBLAS's thread count in this process — the split of the reference's sgemv that decides which domains its
    tail kernels score (fwav_common.h).  The reference would run here with the same numpy, so its scores follow this
    count; ``FWAV_BLAS_THREADS`` overrides it."""
    global _BLAS_THREADS
    env = os.environ.get("FWAV_BLAS_THREADS")
    if env:
        return max(1, int(env))
    if _BLAS_THREADS is None:
        n = None
        try:
            import threadpoolctl
            for info in threadpoolctl.threadpool_info():
                if info.get("user_api") == "blas":
                    n = int(info["num_threads"])
                    break
        except Exception:  # noqa: BLE001
            n = None
        _BLAS_THREADS = max(1, n if n else (os.cpu_count() or 1))
    return _BLAS_THREADS


def numpy_topk_row(scores: np.ndarray, k: int) -> np.ndarray:
    """range_candidates_from_embedding_emb (fractal.py:535-541) + pad_candidates (:544-552) on one score row, by the
    reference's own numpy calls."""
    nd = len(scores)
    if k >= nd:
        idx = np.argsort(scores)[::-1]
    else:
        part = np.argpartition(scores, -k)[-k:]
        idx = part[np.argsort(scores[part])[::-1]]
    out = np.full(k, -1, np.int32)
    out[:min(k, len(idx))] = idx[:k]
    return out


_POOL = None
_SLOTS: list = []
_DRIVER = None
_SIDE: dict = {}


def defer(finish, device: torch.device):
    """Run ``finish(stream)`` — the host half of a tie resolution — on the background driver thread, on a side stream
    that first waits for everything queued so far on ``device``'s current stream.  Returns its Future.  One driver
    thread: resolutions run in call order and share the staging buffers."""
    global _DRIVER
    if _DRIVER is None:
        from concurrent.futures import ThreadPoolExecutor
        _DRIVER = ThreadPoolExecutor(1, thread_name_prefix="fwav-ties-driver")
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
            finish(side.cuda_stream)
            side.synchronize()

    return _DRIVER.submit(job)


def _pool():
    """Host threads for numpy's ranking of the exact score rows (argpartition runs outside the GIL; measured on the
    box's 16-CPU share: 8 threads 5.7x one at cfg2 row widths, `profiles/r03/host_tie_cost.log`)."""
    global _POOL
    if _POOL is None:
        from concurrent.futures import ThreadPoolExecutor
        n = int(os.environ.get("FWAV_TIE_THREADS", str(min(8, os.cpu_count() or 1))))
        _POOL = ThreadPoolExecutor(max(1, n), thread_name_prefix="fwav-ties")
    return _POOL


def _slot(i: int, numel: int) -> torch.Tensor:
    """Reusable page-locked staging row i (float32), grown on demand."""
    while len(_SLOTS) <= i:
        _SLOTS.append(None)
    t = _SLOTS[i]
    if t is None or t.numel() < numel:
        t = torch.empty(numel, dtype=torch.float32, pin_memory=True)
        _SLOTS[i] = t
    return t[:numel]


def resolve_rows(rows: torch.Tensor, *, emb: torch.Tensor, n_domains: int, q_offset: int, k: int, threads: int,
                 ranges: torch.Tensor, range_size: int, pool: torch.Tensor, s_clip: float, cand: torch.Tensor,
                 outs: tuple, stream: int) -> None:
    """Rows (local indices, device int32) whose match depends on numpy's tie order: exact score rows in launches of up
    to DEVICE_ROW_BUDGET (fwav_score_rows reads the embedding table once per launch), copied to a ring of page-locked
    row slots (HOST_ROW_BUDGET), numpy's ranking of each row on a host thread pool as soon as it lands, the new
    candidate rows written back to ``cand`` and the affine solve re-run for those rows into ``outs`` =
    (idx, s, o, sym, err).  (cfg4-sized rows, 86.4 M scores: 22 rows 3.5 → 1.1 s against one 256 MB
    double buffer.)"""
    dev = rows.device
    n = rows.numel()
    if n == 0:
        return
    trace = os.environ.get("FWAV_TIES_TRACE")
    t0 = time.perf_counter()
    tw = 0.0
    nd = int(n_domains)
    per = max(1, min(n, DEVICE_ROW_BUDGET // (4 * nd)))     # rows per fwav_score_rows launch
    nslots = max(2, min(n, HOST_ROW_BUDGET // (4 * nd)))   # rows staged on the host at once
    cv = cand.view(-1, k)
    ex = _pool()
    futs = [None] * n
    slot_busy = [None] * nslots  # the future ranking each slot's row
    S = torch.empty(per * nd, dtype=torch.float32, device=dev)
    ev = torch.cuda.Event()
    for b0 in range(0, n, per):
        rb = rows[b0:b0 + per].contiguous()
        m = rb.numel()
        call("fwav_score_rows", emb.data_ptr(), nd, rb.data_ptr(), m, int(q_offset), int(threads), S.data_ptr(),
             stream)
        # copy the launch's rows to free staging slots in runs of at most nslots, one synchronisation per run
        for r0 in range(0, m, nslots):
            run = range(b0 + r0, b0 + min(m, r0 + nslots))
            hs = []
            for i in run:
                sl = i % nslots
                if slot_busy[sl] is not None:  # its previous row is still being ranked
                    slot_busy[sl].result()
                h = _slot(sl, nd)
                h.copy_(S[(i - b0) * nd:(i - b0 + 1) * nd], non_blocking=True)
                hs.append((i, sl, h))
            ev.record()
            tw0 = time.perf_counter()
            ev.synchronize()
            tw += time.perf_counter() - tw0
            for i, sl, h in hs:
                futs[i] = slot_busy[sl] = ex.submit(numpy_topk_row, h.numpy(), k)
    t1 = time.perf_counter()
    newc = torch.from_numpy(np.stack([f.result() for f in futs])).to(dev)
    if trace:
        print(f"fwav.ties: {n} rows x {nd}: {(time.perf_counter() - t0) * 1e3:.1f} ms (device score rows + copies "
              f"waited {tw * 1e3:.1f} ms, numpy tail {(time.perf_counter() - t1) * 1e3:.1f} ms)", flush=True)
    ridx = rows.long()
    cv[ridx] = newc
    rs = int(range_size)
    rsub = ranges.view(-1, rs)[ridx].contiguous()
    tmp = [torch.empty(n, dtype=t.dtype, device=dev) for t in outs]
    call("fwav_affine", rsub.data_ptr(), n, rs, newc.data_ptr(), k, pool.data_ptr(), nd, float(s_clip),
         *[t.data_ptr() for t in tmp], stream)
    for t, u in zip(outs, tmp):
        t[ridx] = u
