"""Device pipeline: the hot path of ``compress_audio`` / ``decompress_audio`` on one MI355X.

Everything between the input signal and the match arrays stays in HBM and runs on one HIP stream through
the C-ABI of ``libfwav.so`` (``include/fwav.h``); torch only provides device memory and the stream.  There
is no CPU fallback: without the library or a device every call raises :class:`~fwav._lib.FwavError`.

Reference map (``/root/reference/fractal.py``):
  voiced_detection :880-909 + range formation :1074-1112  → fwav_voiced_ranges
  silent-input test :1083                                  → fwav_weighted_energy (f64 partials)
  build_domains_memmap :285-334 + build_domain_embeddings :238-280 → fwav_pool_embed
  cpu_worker energy prune :601-603, pad :622               → fwav_prune
  linear top-K :535-541, 617-620                           → fwav_sim_topk (+ fwav_tie_check / fwav.ties for exact ties)
  _process_gpu_batch :757-850                              → fwav_affine
  decompress_audio :1378-1473                              → fwav_decode
"""
from __future__ import annotations

import dataclasses
import math
from typing import Optional

import numpy as np
import torch

from . import _lib, ties as _ties
from .nporder import zero_query_candidates  # noqa: F401  (Q11 rows; re-exported)
from ._lib import FwavError, call, size_call

F32 = np.float32
#: tie_order → fwav_tie_check's exact_sets argument ("index" never calls it)
TIE_MODES = {"numpy": 0, "numpy_sets": 1, "numpy_rows": 2, "index": -1}


from . import geometry  # noqa: E402,F401  range_size, domain_step (fractal.py:1070-1071)


def n_domains_for(n: int, tile_size: int, step: int) -> int:
    return 0 if n < tile_size else (n - tile_size) // step + 1


def require_device(device=None) -> torch.device:
    _lib.lib()
    if not torch.cuda.is_available():
        raise FwavError("no HIP device visible: the fwav engine has no CPU path")
    return torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())


def _stream(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _p(t: Optional[torch.Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


_TABLES: dict = {}


def embed_tables(rs: int, device: torch.device) -> torch.Tensor:
    key = (rs, str(device))
    if key not in _TABLES:
        host = np.zeros(size_call("fwav_embed_tables_size", rs), np.float64)
        call("fwav_embed_tables", rs, host.ctypes.data)
        _TABLES[key] = torch.from_numpy(host).to(device)
    return _TABLES[key]


_ZERO_CAND_DEV: dict = {}


def _zero_cand_device(n_domains: int, top_k: int, device: torch.device) -> torch.Tensor:
    key = (int(n_domains), int(top_k), str(device))
    if key not in _ZERO_CAND_DEV:
        _ZERO_CAND_DEV[key] = torch.from_numpy(zero_query_candidates(n_domains, top_k)).to(device)
    return _ZERO_CAND_DEV[key]


@dataclasses.dataclass
class DeviceCompressed:
    """Result of :func:`compress_device`.  Device tensors (final once ``wait()`` returns)."""

    n_ranges: int
    range_size: int
    tile_size: int
    domain_step: int
    energy_thresh: float
    original_len: int
    n_domains: int
    top_k: int
    shard: tuple[int, int]
    ranges: Optional[torch.Tensor] = None
    pool: Optional[torch.Tensor] = None
    emb: Optional[torch.Tensor] = None
    cand: Optional[torch.Tensor] = None
    idx: Optional[torch.Tensor] = None
    s: Optional[torch.Tensor] = None
    o: Optional[torch.Tensor] = None
    sym: Optional[torch.Tensor] = None
    err: Optional[torch.Tensor] = None
    n_active: Optional[torch.Tensor] = None
    energy_partial: Optional[torch.Tensor] = None
    ties: Optional[torch.Tensor] = None  # fwav_sim_topk's tie list (keep_intermediates)
    resolved: Optional[torch.Tensor] = None  # local rows re-ranked with numpy's order (keep_intermediates)
    search_ws: Optional[torch.Tensor] = None  # fwav_sim_topk's workspace after the call (keep_intermediates, one launch)
    n_ties: int = 0          # queries whose top K + 1 scores hold exact ties
    n_resolved: int = 0      # of those, rows re-ranked with numpy's own tie order (fwav.ties)
    empty: bool = False
    pending: Optional[object] = None  # deferred tie resolution (compress_device(defer_ties=True)): a Future
    apply: Optional[object] = None    # ... and its last step, run by wait() on the call's own stream
    stream: Optional[object] = None   # the torch stream the call's kernels were queued on

    def wait(self) -> "DeviceCompressed":
        """Complete a deferred tie resolution (no-op otherwise); the outputs are final afterwards.  The fix-up runs on
        the call's own stream, after its search and affine solve, and whichever stream is current here waits for it
        (so both the call's stream and the caller's see final outputs)."""
        if self.pending is not None:
            staged = self.pending.result()
            self.pending = None
            if staged is not None and self.apply is not None:
                st = self.stream if self.stream is not None else torch.cuda.current_stream()
                caller = torch.cuda.current_stream(st.device)
                with torch.cuda.device(st.device), torch.cuda.stream(st):
                    self.apply(*staged)
                if caller != st:
                    ev = torch.cuda.Event()
                    ev.record(st)
                    caller.wait_event(ev)
            self.apply = None
        return self

    def is_silent(self) -> bool:
        """np.sum((signal·mask)²) < 1e-8 (fractal.py:1083): the device computes numpy's float32 sum bit-exactly, and the
        comparison is float32 against float32(1e-8) (NEP 50)."""
        if self.energy_partial is None:
            return True
        return bool(F32(self.energy_partial.cpu().numpy()[0]) < F32(1e-8))


def _mark(ev, name: str, end: bool = False):
    """Record a HIP event on the current stream into ev[name] = [start, end] (bench instrumentation)."""
    if ev is None:
        return
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    ev.setdefault(name, []).append(e)


def _empty(n, rs, tile, step, thr, k) -> DeviceCompressed:
    return DeviceCompressed(0, rs, tile, step, thr, n, 0, k, (0, 0), empty=True)


def _voiced_ranges(sig, n, rs, frame, thr32, lo32, st) -> torch.Tensor:
    """fwav_voiced_ranges on the stream ``st``: the voiced-masked, reflect-padded ranges f32[nr·rs]."""
    nr = -(-n // rs)
    ws_n = size_call("fwav_voiced_workspace_size", n, frame)
    ws = torch.empty(ws_n, dtype=torch.uint8, device=sig.device)
    ranges = torch.empty(nr * rs, dtype=torch.float32, device=sig.device)
    call("fwav_voiced_ranges", sig.data_ptr(), n, rs, frame, 5, float(thr32), float(lo32), ranges.data_ptr(), nr,
         None, ws.data_ptr(), ws_n, st)
    return ranges


def ranges_device(sig: torch.Tensor, tile_size: int, energy_thresh: float = 1e-4) -> tuple[torch.Tensor, int, int]:
    """The ranges alone (voiced detection + range formation, fractal.py:880-909, 1074-1112) on the current stream of
    ``sig``'s device: (ranges f32[nr·rs], nr, rs) — what fwav.dist needs to balance the shards before a compress."""
    if sig.dim() != 1 or sig.dtype != torch.float32 or not sig.is_cuda:
        raise ValueError("ranges_device expects a 1-D float32 device tensor")
    with torch.cuda.device(sig.device):
        sig = sig.contiguous()
        n = sig.numel()
        rs, _ = geometry(tile_size)
        if n == 0:
            raise ValueError("a cannot be empty")
        r = _voiced_ranges(sig, n, rs, 2 * rs, F32(energy_thresh), F32(energy_thresh * 0.5), _stream(sig.device))
        return r, -(-n // rs), rs


def compress_device(sig: torch.Tensor, *args, **kwargs) -> DeviceCompressed:
    """Run the compress hot path on ``sig``'s device (made current for the call: the C ABI's per-device plans and
    kernel attributes are taken from the current HIP device).  See :func:`_compress_device`."""
    with torch.cuda.device(sig.device):
        return _compress_device(sig, *args, **kwargs)


def _compress_device(sig: torch.Tensor, tile_size: int, top_k: int, energy_thresh: float = 1e-4,
                     fast_mode: bool = True, s_clip: float = 16.0, shard: Optional[tuple[int, int]] = None,
                     keep_intermediates: bool = False, events: Optional[dict] = None,
                     search: str = "f16", on_pool=None, blas_threads: Optional[int] = None,
                     tie_order: str = "numpy", defer_ties: bool = False,
                     sub_blocks: Optional[int] = None) -> DeviceCompressed:
    """Run the compress hot path on ``sig`` (1-D float32 tensor on a HIP device).

    ``shard=(lo, hi)`` restricts candidate search and the affine solve to ranges ``[lo, hi)`` (the
    multi-GPU path; a callable ``shard(ranges, n_ranges, range_size) -> (lo, hi)`` picks them once the voiced-masked
    ranges exist); voiced detection, pool and embeddings are always computed for the whole signal,
    because query vectors are domain-embedding rows (quirk Q1) and the voiced state is a scan over the
    whole signal.  Raises ValueError for the reference's own error cases (empty input; n_ranges >
    n_domains).  ``on_pool(pool)``, when given, is called right after the pool kernel is queued (the API
    starts the pool's device→host copy there, on a side stream, so that it overlaps the search).
    ``blas_threads``: the OpenBLAS thread count whose sgemv order the scores follow (default: this process's,
    fwav.ties.blas_threads).  ``tie_order="numpy"`` re-ranks the rows whose match depends on the order of exactly
    equal scores with numpy's own calls, as the reference does (one host synchronisation to read the count), so every
    match tuple is the reference's; ``"numpy_sets"`` also re-ranks every row with a tie at the K-th place, so that
    the candidate sets are the reference's too; ``"numpy_rows"`` re-ranks every row with any exact tie in its top K + 1,
    so that every candidate row, order included, is the reference's (a parity mode: thousands of host rows at cfg2);
    ``"index"`` keeps the device's (score desc, index asc) order (no
    synchronisation).  ``defer_ties=True`` hands that host step to a background thread (its device work on a side
    stream, after this call's kernels) and returns at once: the outputs are final after ``result.wait()``, so a
    stream of calls overlaps one call's host ranking with the next call's search.  Without deferral, a large search
    over a large table runs as ``sub_blocks`` launches over consecutive slices of the active list (default
    :func:`_tie_sub_blocks`), and each slice's tied rows are ranked on the host while the next slice searches.
    """
    if sig.dim() != 1 or sig.dtype != torch.float32 or not sig.is_cuda:
        raise ValueError("compress_device expects a 1-D float32 device tensor")
    dev = sig.device
    st = _stream(dev)
    sig = sig.contiguous()
    n = sig.numel()
    k = int(top_k)
    rs, step = geometry(tile_size)
    frame = 2 * rs
    if n == 0:
        raise ValueError("a cannot be empty")  # np.convolve on zero frames (fractal.py:895)
    nf = -(-n // frame)
    nr = -(-n // rs)
    nd = n_domains_for(n, tile_size, step)
    thr32 = F32(energy_thresh)
    lo32 = F32(energy_thresh * 0.5)
    if k > size_call("fwav_topk_max_k"):
        raise ValueError(f"top_k={k} > {size_call('fwav_topk_max_k')} is not supported by the HIP search")
    if tie_order not in TIE_MODES:
        raise ValueError("tie_order must be 'numpy' (the reference's order of exactly tied scores wherever it decides a"
                         " match), 'numpy_sets' (and wherever it decides a candidate set), 'numpy_rows' (and wherever it"
                         " decides a candidate row's order) or 'index'")
    threads = _ties.blas_threads() if blas_threads is None else int(blas_threads)
    _mark(events, "voiced_ranges")
    ranges = _voiced_ranges(sig, n, rs, frame, thr32, lo32, st)
    partial = torch.empty(1, dtype=torch.float32, device=dev)
    wse = size_call("fwav_weighted_energy_workspace_size", n)
    wsen = torch.empty(wse, dtype=torch.uint8, device=dev)
    call("fwav_weighted_energy", ranges.data_ptr(), n, partial.data_ptr(), wsen.data_ptr(), wse, st)
    _mark(events, "voiced_ranges")
    res = DeviceCompressed(nr, rs, tile_size, step, energy_thresh, n, nd, k, (0, nr), energy_partial=partial,
                           stream=torch.cuda.current_stream(dev))
    if n < tile_size or nr > nd:
        # the reference returns the empty tuple for silent input before it ever builds domains
        if res.is_silent() or n < tile_size:
            return _empty(n, rs, tile_size, step, energy_thresh, k)
        raise ValueError("mmap length is greater than file size")  # quirk Q9 (fractal.py:1190-1195)
    tab = embed_tables(rs, dev)
    pool = torch.empty(nd * rs, dtype=torch.float32, device=dev)
    emb = torch.empty(nd * 16, dtype=torch.float32, device=dev)
    if search not in ("f16", "f32"):
        raise ValueError("search must be 'f16' (fp16 pre-filter + exact f32 rescoring) or 'f32'")
    emb16 = torch.empty(2 * ((nd + 255) // 256) * 256 * 16, dtype=torch.float16, device=dev) if search == "f16" else None
    ws_p = size_call("fwav_pool_workspace_size", n, tile_size, rs, step)
    wsp = torch.empty(max(ws_p, 16), dtype=torch.uint8, device=dev)
    _mark(events, "pool_embed")
    call("fwav_pool_embed", sig.data_ptr(), n, tile_size, rs, step, tab.data_ptr(), pool.data_ptr(), emb.data_ptr(),
         _p(emb16), wsp.data_ptr(), ws_p, st)
    _mark(events, "pool_embed")
    if on_pool is not None:
        on_pool(pool)
    # multi-GPU: bounds chosen from the ranges themselves (fwav.dist balances the prune); evaluated after the pool and
    # embedding kernels are queued, so its host synchronisation overlaps them
    if callable(shard):
        shard = shard(ranges, nr, rs)
    lo, hi = (0, nr) if shard is None else (int(shard[0]), int(shard[1]))
    if not (0 <= lo <= hi <= nr):
        raise ValueError(f"bad shard {shard} for {nr} ranges")
    res.shard = (lo, hi)
    m = hi - lo
    cand = torch.empty(max(m, 1) * k, dtype=torch.int32, device=dev)
    active = torch.empty(max(m, 1), dtype=torch.int32, device=dev)
    n_active = torch.empty(1, dtype=torch.int32, device=dev)
    rsh = ranges[lo * rs:hi * rs]
    idx = torch.empty(m, dtype=torch.int32, device=dev)
    s = torch.empty(m, dtype=torch.float32, device=dev)
    o = torch.empty(m, dtype=torch.float32, device=dev)
    sym = torch.empty(m, dtype=torch.uint8, device=dev)
    err = torch.empty(m, dtype=torch.float32, device=dev)
    if m > 0:
        _mark(events, "prune")
        zc = _zero_cand_device(nd, k, dev)
        call("fwav_prune", rsh.data_ptr(), m, lo, rs, float(F32(energy_thresh * 0.75)), int(bool(fast_mode)),
             emb.data_ptr(), nd, k, zc.data_ptr(), cand.data_ptr(), active.data_ptr(), n_active.data_ptr(), st)
        _mark(events, "prune")
        sc = float(abs(F32(s_clip)))
        nsub = 1
        sliced = False
        if tie_order != "index":
            if sub_blocks is not None:
                nsub = int(sub_blocks)
            elif not defer_ties or nd >= SUB_BLOCK_MIN_DOMAINS:
                nsub = _tie_sub_blocks(m, nd)
            nsub = max(1, min(nsub, m))
            # large tables, deferred: the sliced path too (even as one slice), so that the exact score rows are
            # queued right after the search instead of behind the next call's (the driver thread's side stream
            # would wait for it), and only the copies, numpy's ranking and the fix-up are deferred
            sliced = nsub > 1 or (defer_ties and nd >= SUB_BLOCK_MIN_DOMAINS)
        if not sliced:
            _mark(events, "sim_topk")
            wk = size_call("fwav_sim_topk_workspace_size", m, nd, k) if (emb16 is not None or k > 64) else 0
            wsk = torch.empty(max(wk, 16), dtype=torch.uint8, device=dev)
            ties = (torch.empty(size_call("fwav_tie_list_size", m), dtype=torch.int32, device=dev)
                    if tie_order != "index" else None)
            call("fwav_sim_topk", emb.data_ptr(), _p(emb16), nd, active.data_ptr(), n_active.data_ptr(), m, lo, k,
                 threads, cand.data_ptr(), _p(ties), wsk.data_ptr(), wk, st)
            _mark(events, "sim_topk")
            _mark(events, "affine")
            call("fwav_affine", rsh.data_ptr(), m, rs, cand.data_ptr(), k, pool.data_ptr(), nd, sc, idx.data_ptr(),
                 s.data_ptr(), o.data_ptr(), sym.data_ptr(), err.data_ptr(), st)
            _mark(events, "affine")
        if not sliced and ties is not None:
            # exactly tied scores whose order can change a match: numpy's own ranking for those rows (fwav.ties)
            _mark(events, "ties")
            resolve = torch.empty(m + 1, dtype=torch.int32, device=dev)
            call("fwav_tie_check", rsh.data_ptr(), m, rs, cand.data_ptr(), k, pool.data_ptr(), nd, emb.data_ptr(), lo,
                 threads, ties.data_ptr(), m, TIE_MODES[tie_order], resolve.data_ptr(), st)

            def finish(stream_id):
                counts = torch.stack([ties[0], resolve[0]]).cpu()
                res.n_ties, res.n_resolved = int(counts[0]), int(counts[1])
                if res.n_resolved:
                    _ties.resolve_rows(resolve[1:1 + res.n_resolved], emb=emb, n_domains=nd, q_offset=lo, k=k,
                                       threads=threads, ranges=rsh, range_size=rs, pool=pool, s_clip=sc, cand=cand,
                                       outs=(idx, s, o, sym, err), stream=stream_id)

            def stage(stream_id):
                # deferred: on the driver thread, the counts, the exact score rows and their copies; numpy's ranking
                # then runs on the host pool while the driver moves on to the next call, and wait() applies it
                counts = torch.stack([ties[0], resolve[0]]).cpu()
                res.n_ties, res.n_resolved = int(counts[0]), int(counts[1])
                if not res.n_resolved:
                    return None
                rows = resolve[1:1 + res.n_resolved]
                futs = _ties.rank_rows(_ties.score_row_launches(rows, emb=emb, n_domains=nd, q_offset=lo,
                                                                threads=threads, stream=stream_id),
                                       res.n_resolved, nd, k)
                return rows, futs

            def apply(rows, futs):
                _ties.apply_rows(rows, futs, ranges=rsh, range_size=rs, pool=pool, n_domains=nd, k=k, s_clip=sc,
                                 cand=cand, outs=(idx, s, o, sym, err), stream=_stream(dev))

            if defer_ties:
                res.apply = apply
                res.pending = _ties.defer(stage, dev)
            else:
                finish(st)
                if keep_intermediates:
                    res.resolved = resolve[1:1 + res.n_resolved]
            _mark(events, "ties")
        elif sliced:
            ties = _search_sub_blocks(nsub, m, nd, k, lo, rs, threads, sc, tie_order, emb, emb16, active, n_active,
                                      rsh, pool, cand, (idx, s, o, sym, err), res, events, st, defer=defer_ties)
    res.pool, res.idx, res.s, res.o, res.sym, res.err, res.n_active = pool, idx, s, o, sym, err, n_active
    if keep_intermediates:
        res.ranges, res.emb, res.cand, res.active = ranges, emb, cand, active
        if m > 0 and ties is not None:
            res.ties = ties
        if m > 0 and not sliced:
            res.search_ws = wsk
    return res


#: query sub-blocks of a search whose tied rows are ranked while the next sub-block searches: only where numpy's
#: ranking of a row is expensive (tables of ≥ 4 Mi domains: a cfg3 row 13 ms, a cfg4 row ≈ 50 ms on the host) and
#: every sub-block still fills the chip for a few rounds (≥ 400,000 queries; a slice launch costs ≈ 26 ms more at
#: cfg3, 60 ms at cfg4: profiles/r03/sub_blocks_cfg3.log, sub_blocks_cfg4_eighth.log)
SUB_BLOCK_MIN_DOMAINS = 1 << 22
TIE_REC = 9  # int32 per tie record (kTieRec, fwav_common.h)
SUB_BLOCK_QUERIES = 400_000


def _tie_sub_blocks(m: int, nd: int) -> int:
    if nd < SUB_BLOCK_MIN_DOMAINS:
        return 1
    return max(1, min(8, m // SUB_BLOCK_QUERIES))


def _slice_bounds(m: int, nsub: int) -> list[tuple[int, int]]:
    """Consecutive slices [a, b) of m active-list positions, the last one half-size: its tied rows are the only ones
    ranked after the search has ended."""
    nsub = max(1, min(int(nsub), m))
    wts = [2] * (nsub - 1) + [1]
    cuts = [m * sum(wts[:j]) // sum(wts) for j in range(nsub + 1)]
    return [(cuts[j], cuts[j + 1]) for j in range(nsub) if cuts[j + 1] > cuts[j]]


class _Staged:
    """A deferred sliced tie resolution: the slices' (rows, future of their ranking) pairs (DeviceCompressed.wait)."""

    def __init__(self, pend):
        self.pend = pend

    def result(self):
        return (self.pend,)


def _search_sub_blocks(nsub, m, nd, k, lo, rs, threads, sc, tie_order, emb, emb16, active, n_active, rsh, pool, cand,
                       outs, res, events, st, defer=False):
    """The search as ``nsub`` launches over consecutive slices of the active list.  After each slice's search and tie
    check the host reads its tie counts (one synchronisation), queues the exact score rows of its tied rows and hands
    their copies and numpy's ranking to the driver thread (fwav.ties.rank_rows_async); then the next slice searches.
    The affine solve runs once over the shard after the last slice, then the ranked rows are applied.  Returns the
    slices' tie records as one list."""
    dev = rsh.device
    bounds = _slice_bounds(m, nsub)
    wk = max(size_call("fwav_sim_topk_workspace_size", b - a, nd, k) for a, b in bounds) \
        if (emb16 is not None or k > 64) else 0
    wsk = torch.empty(max(wk, 16), dtype=torch.uint8, device=dev)
    pend = []
    lists = []  # each slice's tie records
    n_ties = n_res = 0
    _mark(events, "sim_topk")
    for j0, j1 in bounds:
        mq = j1 - j0
        na = torch.clamp(n_active - j0, 0, mq).to(torch.int32)
        ties = torch.empty(size_call("fwav_tie_list_size", mq), dtype=torch.int32, device=dev)
        call("fwav_sim_topk", emb.data_ptr(), _p(emb16), nd, active[j0:].data_ptr(), na.data_ptr(), mq, lo, k, threads,
             cand.data_ptr(), ties.data_ptr(), wsk.data_ptr(), wk, st)
        resolve = torch.empty(mq + 1, dtype=torch.int32, device=dev)
        call("fwav_tie_check", rsh.data_ptr(), m, rs, cand.data_ptr(), k, pool.data_ptr(), nd, emb.data_ptr(), lo,
             threads, ties.data_ptr(), mq, TIE_MODES[tie_order], resolve.data_ptr(), st)
        counts = torch.stack([ties[0], resolve[0]]).cpu()
        if _ties._TRACE:
            import time
            print(f"fwav.engine {time.perf_counter():.4f}: slice {j0}..{j1} searched, {int(counts[1])} tied rows",
                  flush=True)
        n_ties += int(counts[0])
        lists.append(ties[1:1 + TIE_REC * int(counts[0])])
        nr_j = int(counts[1])
        n_res += nr_j
        if nr_j:
            rows = resolve[1:1 + nr_j]
            pend.append((rows, _ties.rank_rows_async(rows, emb=emb, n_domains=nd, q_offset=lo, k=k, threads=threads,
                                                     stream=st)))
    _mark(events, "sim_topk")
    _mark(events, "affine")
    call("fwav_affine", rsh.data_ptr(), m, rs, cand.data_ptr(), k, pool.data_ptr(), nd, sc, *[t.data_ptr() for t in outs],
         st)
    _mark(events, "affine")
    def apply(pend_):
        for rows, fut in pend_:
            _ties.apply_rows(rows, fut.result(), ranges=rsh, range_size=rs, pool=pool, n_domains=nd, k=k, s_clip=sc,
                             cand=cand, outs=outs, stream=_stream(dev))

    res.n_ties, res.n_resolved = n_ties, n_res
    res.resolved = torch.cat([r for r, _ in pend]) if pend else torch.empty(0, dtype=torch.int32, device=dev)
    if defer:  # wait() applies the rankings on the caller's stream
        res.pending, res.apply = _Staged(pend), apply
    else:
        _mark(events, "ties")
        apply(pend)
        _mark(events, "ties")
    # one tie list in fwav_sim_topk's layout (count, then the records of every slice)
    return torch.cat([torch.tensor([n_ties], dtype=torch.int32, device=dev)] + lists)


def decompress_device(idx: torch.Tensor, *args, **kwargs):
    """decompress_audio's loop on ``idx``'s device (made current for the call).  See :func:`_decompress_device`."""
    with torch.cuda.device(idx.device):
        return _decompress_device(idx, *args, **kwargs)


def _decompress_device(idx: torch.Tensor, s: torch.Tensor, o: torch.Tensor, sym: torch.Tensor, pool: torch.Tensor,
                       n_ranges: int, range_size: int, iterations: int = 8, convergence_eps: float = 1e-3,
                       s_clip: float = 16.0, s_damping: float = 0.0):
    """decompress_audio's loop on device.  Returns (recon f32[n_ranges*range_size] tensor, iterations_run,
    deltas f64 list).  One host synchronisation (to read the iteration count and the result buffer), plus one per
    early-exit check: where the f64 Δ cannot decide the reference's Δ < eps (fractal.py:1460-1465), fwav_decode stops
    for fwav_decode_exact (the reference's own sdot order) and the loop resumes when the reference goes on."""
    dev = idx.device
    st = _stream(dev)
    nr, rs = int(n_ranges), int(range_size)
    nd = pool.numel() // rs if rs > 0 else 0
    it = int(iterations)
    eps = float(convergence_eps)
    a = torch.empty(max(nr * rs, 1), dtype=torch.float32, device=dev)
    b = torch.empty(max(nr * rs, 1), dtype=torch.float32, device=dev)
    deltas = torch.zeros(max(it, 1), dtype=torch.float64, device=dev)
    state = torch.zeros(4, dtype=torch.int32, device=dev)
    wsn = size_call("fwav_decode_workspace_size", nr, rs, it)
    ws = torch.empty(max(wsn, 16), dtype=torch.uint8, device=dev)
    done, init, out = 0, None, a
    while True:
        call("fwav_decode_from", idx.data_ptr(), s.data_ptr(), o.data_ptr(), sym.data_ptr(), nr, rs, pool.data_ptr(),
             nd, it - done, eps, float(abs(F32(s_clip))), float(s_damping), _p(init), a.data_ptr(), b.data_ptr(),
             deltas[done:].data_ptr(), state.data_ptr(), ws.data_ptr(), wsn, st)
        stt = state.cpu().numpy()
        ran = int(stt[1])
        out, other = (b, a) if int(stt[2]) == 1 else (a, b)
        if int(stt[0]) == 2:  # the reference's Δ decides: computed in its own sdot order
            call("fwav_decode_exact", other.data_ptr(), out.data_ptr(), nr * rs, eps, ran - 1,
                 deltas[done:].data_ptr(), state.data_ptr(), st)
            if int(state[0].item()) == 3 and done + ran < it:  # it goes on: resume from this reconstruction
                init = out.clone()
                done += ran
                continue
        done += ran
        break
    if nr == 0:
        out = a[:0]
    return out[:nr * rs], done, deltas.cpu().numpy()[:done].tolist()
