"""Multi-GPU compress and decompress of ONE signal, ranges sharded across ranks (one process per GPU,
torch.distributed; backend "nccl" is RCCL over xGMI on ROCm).

Compress (reference split ``np.array_split`` of ranges over workers, fractal.py:1180-1182):
  1. rank 0 holds the signal; ONE broadcast of the raw signal (f32, 4 B/sample: 691 MB at cfg4).  Broadcasting
     the signal instead of the domain pool (2.76 GB at cfg4) moves 4× fewer bytes and is sufficient: every rank
     rebuilds voiced mask, ranges, pool and embeddings bit-identically in a few ms (the ranges need the signal and
     the voiced-state scan over the whole signal, so the pool alone would not do);
  2. every rank computes the same contiguous range blocks, balanced by the ranges that survive the energy prune
     (mean(r²) of the voiced-masked ranges the search will actually see; silent stretches cost nothing);
  3. each rank searches + solves its block; the SoA match arrays (17 B/range) are gathered to rank 0, the only
     rank that writes the .fwav.  No collective runs inside the search.

Decompress (cfg5; fractal.py:1378-1473): rank 0 broadcasts the pool and scatters the match arrays; each rank runs
the iteration-resident decode kernel on its ranges; per chunk of up to 64 iterations the ranks all-reduce the
per-block Δ partials (a few hundred KB) and take the same early-exit decision; the reconstruction is gathered to
rank 0.  Shard bounds are multiples of ``fwav_decode_span()`` ranges, so Δ, the iteration count and the output
are bit-identical to the single-GPU decode at any world size (fwav_decode.hip header).  Where the f64 Δ cannot decide
the reference's Δ < eps for certain, every rank stops for the check: the two reconstructions around that iteration
are gathered to rank 0, which computes the reference's Δ in its own sdot order (fwav_decode_exact) and broadcasts
the decision, and the ranks resume from their slices when the reference goes on.

Collectives run on device tensors with RCCL and on host tensors with gloo (CPU tests, and the one-GPU rehearsal
where ranks share cuda:0).  The per-rank compute is pluggable (``compute`` / ``decoder``) so the communication
code is exercised on CPU in tests; the product defaults are the HIP engine on the rank's GPU.
"""
from __future__ import annotations

import time
from typing import Callable, Optional

import numpy as np
import torch
import torch.distributed as dist

from .engine import geometry

FIELDS = ("idx", "s", "o", "sym", "err")


# ------------------------------------------------------------------------------------------------ helpers
#: longest range the range-sharded decode keeps in registers (fwav_decode.hip kMaxResidentRs)
RESIDENT_MAX_RS = 32

def _coll_device(group, device: torch.device) -> torch.device:
    """Where collective buffers live: the GPU for RCCL, the host for gloo."""
    return device if dist.get_backend(group) == "nccl" else torch.device("cpu")


def _broadcast_(t: torch.Tensor, group, device: torch.device) -> torch.Tensor:
    cd = _coll_device(group, device)
    if t.device == cd:
        dist.broadcast(t, src=0, group=group)
        return t
    buf = t.to(cd)
    dist.broadcast(buf, src=0, group=group)
    t.copy_(buf)
    return t


_SIDE: dict = {}


def _side_stream(device: torch.device):
    key = str(device)
    if key not in _SIDE:
        _SIDE[key] = torch.cuda.Stream(device)
    return _SIDE[key]


def _sync(device: torch.device) -> None:
    if device.type == "cuda":
        torch.cuda.synchronize(device)


def balanced_bounds(weights: np.ndarray, world: int) -> list[tuple[int, int]]:
    """Contiguous blocks of len(weights) items with ~equal total weight (every item weight >= a floor so
    all-zero stretches still split evenly)."""
    n = len(weights)
    w = np.asarray(weights, np.float64) + 1e-3
    cs = np.concatenate([[0.0], np.cumsum(w)])
    cuts = [0] + [int(np.searchsorted(cs, cs[-1] * r / world, side="left")) for r in range(1, world)] + [n]
    cuts = np.maximum.accumulate(np.clip(cuts, 0, n))
    return [(int(cuts[r]), int(cuts[r + 1])) for r in range(world)]


def prune_balanced_bounds(ranges: torch.Tensor, n_ranges: int, range_size: int, energy_thresh: float,
                          world: int) -> list[tuple[int, int]]:
    """Range blocks balanced by the energy prune of cpu_worker (fractal.py:601-603): a range whose voiced-masked
    mean(r²) clears float32(0.75·thr) costs one full-table search (weight 1024), a pruned one almost nothing
    (weight 1).  Integer weights and an integer cumsum, so every rank derives the same bounds from its own
    (bit-identical) ranges with no collective.  Scheduling only: the exact prune runs inside each rank's search."""
    if world == 1 or n_ranges == 0:
        return [(0, n_ranges)] + [(n_ranges, n_ranges)] * (world - 1)
    x = ranges[:n_ranges * range_size].view(n_ranges, range_size)
    thr = float(np.float32(energy_thresh * 0.75))
    active = (x.double().square().mean(dim=1) >= thr).to(torch.int64)
    cs = torch.cumsum(active * 1023 + 1, dim=0)
    # targets total·r // world on the device: one host synchronisation (the cut positions)
    r = torch.arange(1, world, dtype=torch.int64, device=cs.device)
    targets = torch.div(cs[-1] * r, world, rounding_mode="floor")
    cuts = torch.searchsorted(cs, targets, right=True).cpu().tolist()
    cuts = [0] + [min(int(c), n_ranges) for c in cuts] + [n_ranges]
    cuts = np.maximum.accumulate(cuts)
    return [(int(cuts[r]), int(cuts[r + 1])) for r in range(world)]


def _pack(fields: dict, length: int, device) -> torch.Tensor:
    out = torch.zeros((5, length), dtype=torch.int32, device=device)
    m = len(fields["idx"])
    out[0, :m] = fields["idx"].to(device=device, dtype=torch.int32)
    out[1, :m] = fields["s"].to(device).view(torch.int32)
    out[2, :m] = fields["o"].to(device).view(torch.int32)
    out[3, :m] = fields["sym"].to(device=device, dtype=torch.int32)
    out[4, :m] = fields["err"].to(device).view(torch.int32)
    return out


def _unpack(packed: torch.Tensor, blocks) -> dict:
    parts = {f: [] for f in FIELDS}
    for r, (a, b) in enumerate(blocks):
        m = b - a
        p = packed[r]
        parts["idx"].append(p[0, :m])
        parts["s"].append(p[1, :m].view(torch.float32))
        parts["o"].append(p[2, :m].view(torch.float32))
        parts["sym"].append(p[3, :m].to(torch.uint8))
        parts["err"].append(p[4, :m].view(torch.float32))
    return {f: torch.cat(v) for f, v in parts.items()}


# ------------------------------------------------------------------------------------------------ compress
def _device_compute(sig, tile_size, top_k, energy_thresh, shard):
    from .engine import compress_device
    r = compress_device(sig, tile_size, top_k, energy_thresh=energy_thresh, shard=shard)
    if r.empty:
        return None
    return dict(idx=r.idx, s=r.s, o=r.o, sym=r.sym, err=r.err, pool=r.pool, n_ranges=r.n_ranges,
                n_domains=r.n_domains, silent=r.is_silent)


def compress_sharded_device(sig: Optional[torch.Tensor], tile_size: int, top_k: int, energy_thresh: float = 1e-4,
                            group=None, device: Optional[torch.device] = None, compute: Optional[Callable] = None,
                            timings: Optional[dict] = None, n: Optional[int] = None):
    """The sharded compress on device tensors.  ``sig`` (1-D f32, on ``device``) is needed on rank 0 only.
    Returns on rank 0 a dict of full-length device tensors idx/s/o/sym/err, the pool, the blocks and geometry, and
    ``is_silent()`` (the reference's silent-input test, one device read); None on the other ranks (``empty=True``
    without arrays for empty / short input).  ``n`` (the signal length, if every rank knows it) saves broadcasting it.
    ``timings`` (if given) receives per-phase host seconds (broadcast / compute / gather), each phase then closed by
    a device synchronisation (without it the phases run back to back, with no synchronisation of their own).
    Equal to ``compress_sharded_finish(compress_sharded_start(...))``."""
    return compress_sharded_finish(compress_sharded_start(sig, tile_size, top_k, energy_thresh, group, device, compute,
                                                          timings, n))


def compress_sharded_start(sig: Optional[torch.Tensor], tile_size: int, top_k: int, energy_thresh: float = 1e-4,
                           group=None, device: Optional[torch.device] = None, compute: Optional[Callable] = None,
                           timings: Optional[dict] = None, n: Optional[int] = None,
                           signal_ready: bool = False) -> dict:
    """First half of :func:`compress_sharded_device`: the signal broadcast and this rank's search + solve, queued.
    ``compute`` may return a ``wait`` callable (a deferred tie resolution, engine.compress_device(defer_ties=True));
    :func:`compress_sharded_finish` calls it before the gather.  A stream of calls can keep a few started calls in
    flight and finish them in order, so that one call's host tie ranking overlaps the next calls' searches (bench.py);
    every rank must start and finish the same calls in the same order (the collectives pair up by order).
    ``signal_ready=True`` (rank 0): ``sig`` is complete on every stream, so the broadcast need not wait for the work
    already queued on the current stream."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    compute = compute or _device_compute
    tm = timings if timings is not None else {}
    timed = timings is not None

    def mark():
        if timed:
            _sync(device)
        return time.perf_counter()

    t0 = time.perf_counter()
    if n is None:
        n_t = torch.zeros(1, dtype=torch.int64, device=device)
        if rank == 0:
            n_t[0] = int(sig.numel())
        _broadcast_(n_t, group, device)
        n = int(n_t.item())
    rs, step = geometry(tile_size)
    blocks_box: list = []
    pre = None
    if device.type == "cuda" and n > 0:
        # Broadcast, ranges and shard bounds on a side stream: the bounds' host synchronisation then waits for these
        # few kernels only, not for the calls still searching on the main stream (a stream of calls keeps the
        # device busy).  The search reads the ranges again on the main stream (a few hundred µs, bit-identical).
        main = torch.cuda.current_stream(device)
        side = _side_stream(device)
        if rank == 0 and not signal_ready:
            side.wait_stream(main)  # the signal may still be in flight on the main stream
        with torch.cuda.stream(side):
            if rank != 0:
                sig = torch.empty(n, dtype=torch.float32, device=device)
            _broadcast_(sig, group, device)  # the one data-path collective before the search
            if world > 1:
                from .engine import ranges_device
                rg, nr_, rs_ = ranges_device(sig, tile_size, energy_thresh)
                pre = prune_balanced_bounds(rg, nr_, rs_, energy_thresh, world)
        main.wait_stream(side)
        sig.record_stream(main)
    else:
        if rank != 0:
            sig = torch.empty(n, dtype=torch.float32, device=device)
        _broadcast_(sig, group, device)  # the one data-path collective before the search
    t1 = mark()

    def shard(ranges, n_ranges, range_size):
        blocks_box[:] = pre if pre is not None else prune_balanced_bounds(ranges, n_ranges, range_size, energy_thresh,
                                                                          world)
        return blocks_box[rank]

    res = compute(sig, tile_size, top_k, energy_thresh, shard)
    return dict(rank=rank, world=world, group=group, device=device, res=res, blocks=blocks_box, n=n, rs=rs,
                step=step, tm=tm, mark=mark, t=[t0, t1])


def compress_sharded_finish(h: dict):
    """Second half of :func:`compress_sharded_device` for a handle from :func:`compress_sharded_start`: completes a
    deferred tie resolution, then gathers the match arrays to rank 0."""
    res, tm, mark = h["res"], h["tm"], h["mark"]
    t0, t1 = h["t"]
    rank, world, group, n, rs, step = h["rank"], h["world"], h["group"], h["n"], h["rs"], h["step"]
    if res is not None and res.get("wait") is not None:
        res["wait"]()
    t2 = mark()
    if res is None:  # empty / short / silent input: identical decision on every rank
        tm.update(broadcast_s=t1 - t0, compute_s=t2 - t1, gather_s=0.0)
        return dict(empty=True, n_ranges=0, range_size=rs, domain_step=step, original_len=n) if rank == 0 else None
    nr = -(-n // rs)
    blocks = h["blocks"]
    maxlen = max(1, max(b - a for a, b in blocks))
    cd = _coll_device(group, h["device"])
    mine = _pack(res, maxlen, cd)
    glist = [torch.empty_like(mine) for _ in range(world)] if rank == 0 else None
    dist.gather(mine, gather_list=glist, dst=0, group=group)
    t3 = mark()
    tm.update(broadcast_s=t1 - t0, compute_s=t2 - t1, gather_s=t3 - t2)
    if rank != 0:
        return None
    out = _unpack(torch.stack(glist), blocks)
    # the silent-input test reads a device value: left to the caller (compress_sharded), so that a stream of calls
    # does not synchronise here with the calls still in flight
    silent = res.get("silent")
    out.update(is_silent=silent if callable(silent) else (lambda: False), n_ranges=nr, range_size=rs,
               domain_step=step, original_len=n, pool=res["pool"], blocks=blocks)
    return out


def compress_sharded(signal: Optional[np.ndarray], tile_size: int, top_k: int, energy_thresh: float = 1e-4,
                     group=None, device: Optional[torch.device] = None, compute: Optional[Callable] = None):
    """Compress one signal with its ranges split across the ranks of ``group``.

    ``signal`` is read on rank 0 only (other ranks may pass None).  Returns, on rank 0, a dict with the
    full SoA match arrays (numpy), ``pool`` (numpy [n_domains, range_size]), n_ranges, range_size,
    domain_step, original_len, and the per-rank blocks; other ranks return None.
    """
    rank = dist.get_rank(group)
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    sig = None
    if rank == 0:
        sig = torch.from_numpy(np.ascontiguousarray(signal, dtype=np.float32)).to(device)
    out = compress_sharded_device(sig, tile_size, top_k, energy_thresh, group, device, compute)
    if rank != 0:
        return None
    if out.get("empty") and "idx" not in out:
        return out
    host = {f: out[f].cpu().numpy() for f in FIELDS}
    host["empty"] = bool(out.pop("is_silent")())
    pool = out["pool"]
    pool = pool.cpu().numpy() if isinstance(pool, torch.Tensor) else np.asarray(pool)
    host.update({k: v for k, v in out.items() if k not in FIELDS and k != "pool"})
    host["pool"] = pool.reshape(-1, out["range_size"])
    return host


# ---------------------------------------------------------------------------------------------- decompress
def decode_beta(n: int) -> float:
    """Relative bound between the reference's float32 Δ (BLAS sdot norms of n values) and the exact one
    (fwav_decode.hip dec_beta)."""
    return 1.01 * ((int(n) + 63) // 64 + 16) * 2.0 ** -24


def decode_decision(rr: float, dd: float, delta: float, eps: float, beta: float) -> int:
    """The device's early-exit decision for the f64 Δ (fwav_decode.hip dec_decide): 1 stop, 0 go on, 2 check."""
    if dd == 0.0:
        return 1 if 0.0 < eps else 0
    if dd < 1e-30 or dd > 1e36 or (rr > 0.0 and (rr < 1e-30 or rr > 1e36)):
        return 2
    b = beta + 1e-7
    if delta * (1.0 + b) < eps:
        return 1
    if delta * (1.0 - b) >= eps:
        return 0
    return 2


def decode_span() -> int:
    from ._lib import size_call
    return size_call("fwav_decode_span")


def decode_bounds(n_ranges: int, world: int, span: Optional[int] = None) -> list[tuple[int, int]]:
    """Contiguous range blocks on multiples of the decode span (the canonical Δ reduction unit), as even as the
    span allows.  Decode cost per range is uniform, so no weighting."""
    span = span or decode_span()
    nb = -(-n_ranges // span)
    out = []
    for r in range(world):
        a = min(n_ranges, (nb * r // world) * span)
        b = min(n_ranges, (nb * (r + 1) // world) * span)
        out.append((a, b))
    return out


class ShardDecoder:
    """One rank's share of the range-sharded decode on its GPU: the C-ABI sequence fwav_decode_run /
    fwav_decode_reduce per chunk and fwav_decode_finish (include/fwav.h).  Everything is queued on the current
    stream; the only host synchronisation is in :meth:`finish`."""

    def __init__(self, idx, s, o, sym, pool, lo, n_ranges_global, range_size, iterations, eps, s_clip=16.0,
                 s_damping=0.0, init: Optional[torch.Tensor] = None):
        from ._lib import size_call
        self.idx, self.s, self.o, self.sym, self.pool = idx, s, o, sym, pool
        self.init = init  # the rank's reconstruction to start from (None: zeros) — a resumed loop
        self.dev = idx.device
        self.m, self.lo, self.nr, self.rs = int(idx.numel()), int(lo), int(n_ranges_global), int(range_size)
        self.nd = pool.numel() // self.rs
        self.iterations, self.eps = int(iterations), float(eps)
        self.s_clip, self.s_damping = float(abs(np.float32(s_clip))), float(s_damping)
        ci = size_call("fwav_decode_chunk_iterations")
        self.n_chunks = size_call("fwav_decode_n_chunks", self.iterations, self.eps)
        self.span = size_call("fwav_decode_span")
        self.n_prefix = ci * (-(-max(self.nr, 1) // self.span)) * 2
        self.partials = torch.zeros(size_call("fwav_decode_partials_count", self.nr), dtype=torch.float64,
                                    device=self.dev)
        self.a = torch.empty(max(self.m * self.rs, 1), dtype=torch.float32, device=self.dev)
        self.b = torch.empty(max(self.m * self.rs, 1), dtype=torch.float32, device=self.dev)
        self.deltas = torch.zeros(max(self.iterations, 1), dtype=torch.float64, device=self.dev)
        self.state = torch.zeros(4, dtype=torch.int32, device=self.dev)

    def _st(self):
        return torch.cuda.current_stream(self.dev).cuda_stream

    def _common(self):
        return (self.idx.data_ptr(), self.s.data_ptr(), self.o.data_ptr(), self.sym.data_ptr(), self.m, self.lo,
                self.nr, self.rs, self.pool.data_ptr(), self.nd, self.iterations)

    def run(self, chunk: int) -> None:
        from ._lib import call
        call("fwav_decode_run", *self._common(), chunk, self.eps, self.s_clip, self.s_damping, self._init(),
             self.a.data_ptr(), self.b.data_ptr(), self.partials.data_ptr(), self.state.data_ptr(), self._st())

    def _init(self):
        return None if self.init is None else self.init.data_ptr()

    def partials_prefix(self) -> torch.Tensor:
        """The block partials the ranks all-reduce (SUM) between run() and reduce()."""
        return self.partials[:self.n_prefix]

    def reduce(self, chunk: int) -> None:
        from ._lib import call
        call("fwav_decode_reduce", self.partials.data_ptr(), self.nr, self.rs, self.iterations, chunk, self.eps,
             self.deltas.data_ptr(), self.state.data_ptr(), self._st())

    def finish(self):
        """→ (local reconstruction f32[m·rs] device tensor, iterations run, deltas list, pending): pending is None,
        or — stopped for the exact check — the local reconstruction before the last iteration (the result is after
        it)."""
        from ._lib import call
        if self.iterations == 0 or self.nr == 0:
            return torch.zeros(self.m * self.rs, dtype=torch.float32, device=self.dev), 0, [], None
        call("fwav_decode_finish", *self._common(), self.eps, self.s_clip, self.s_damping, self._init(),
             self.a.data_ptr(), self.b.data_ptr(), self.state.data_ptr(), self._st())
        st = self.state.cpu().numpy()
        ran = int(st[1])
        out, other = (self.b, self.a) if int(st[2]) == 1 else (self.a, self.b)
        pending = other[:self.m * self.rs] if int(st[0]) == 2 else None
        return out[:self.m * self.rs], ran, self.deltas.cpu().numpy()[:ran].tolist(), pending

    def exact_delta(self, prev: torch.Tensor, nxt: torch.Tensor) -> tuple[float, bool]:
        """Rank 0: the reference's Δ between the whole signal's reconstructions (fwav_decode_exact) and whether it
        stops the loop."""
        from ._lib import call
        st = torch.tensor([2, 0, 0, 0], dtype=torch.int32, device=self.dev)
        d = torch.zeros(1, dtype=torch.float64, device=self.dev)
        prev = prev.to(self.dev).contiguous()
        nxt = nxt.to(self.dev).contiguous()
        call("fwav_decode_exact", prev.data_ptr(), nxt.data_ptr(), prev.numel(), self.eps, 0, d.data_ptr(),
             st.data_ptr(), self._st())
        return float(d.item()), int(st[0].item()) == 1

    def resumed(self, rec: torch.Tensor, iterations_left: int) -> "ShardDecoder":
        """The same shard continuing from its reconstruction ``rec`` for ``iterations_left`` more iterations."""
        return ShardDecoder(self.idx, self.s, self.o, self.sym, self.pool, self.lo, self.nr, self.rs, iterations_left,
                            self.eps, self.s_clip, self.s_damping, init=rec.clone())


def _all_reduce_sum_(t: torch.Tensor, group, device: torch.device) -> None:
    cd = _coll_device(group, device)
    if t.device == cd:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        return
    buf = t.to(cd)
    dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
    t.copy_(buf)


def _gather_to_rank0(t: torch.Tensor, group, device: torch.device) -> Optional[torch.Tensor]:
    """The ranks' local slices (in rank order = signal order) concatenated on rank 0; None elsewhere."""
    cd = _coll_device(group, device)
    n = torch.tensor([t.numel()], dtype=torch.int64, device=cd)
    world = dist.get_world_size(group)
    ns = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    ns = [int(x.item()) for x in ns]
    buf = torch.zeros(max(max(ns), 1), dtype=t.dtype, device=cd)
    buf[:t.numel()] = t.to(cd)
    rank = dist.get_rank(group)
    glist = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, gather_list=glist, dst=0, group=group)
    if rank != 0:
        return None
    return torch.cat([g[:k] for g, k in zip(glist, ns)])


def decode_shard(decoder, group=None, device: Optional[torch.device] = None):
    """Drive one rank's decoder through the chunk loop with the per-chunk all-reduce of Δ partials.  A stop for the
    exact early-exit check (fwav_decode.hip): both reconstructions gathered to rank 0, the reference's Δ there
    (decoder.exact_delta), its decision broadcast, and the loop resumed on every rank when the reference goes on.
    → (local reconstruction, iterations run, deltas)."""
    device = device or decoder.dev
    total = decoder.iterations
    done, deltas = 0, []
    while True:
        for c in range(decoder.n_chunks):
            decoder.run(c)
            _all_reduce_sum_(decoder.partials_prefix(), group, device)
            decoder.reduce(c)
        rec, ran, dl, pending = decoder.finish()
        done += ran
        deltas += dl
        if pending is None:
            return rec, done, deltas
        prev_all = _gather_to_rank0(pending, group, device)
        next_all = _gather_to_rank0(rec, group, device)
        cd = _coll_device(group, device)
        verdict = torch.zeros(2, dtype=torch.float64, device=cd)
        if dist.get_rank(group) == 0:
            d_ref, stop = decoder.exact_delta(prev_all, next_all)
            verdict[0], verdict[1] = d_ref, 1.0 if stop else 0.0
        _broadcast_(verdict, group, device)
        deltas[-1] = float(verdict[0].item())
        if verdict[1].item() != 0.0 or done >= total:
            return rec, done, deltas
        decoder = decoder.resumed(rec, total - done)


def decompress_sharded(matches_soa: Optional[dict], domains: Optional[np.ndarray], n_ranges: int, range_size: int,
                       iterations: int = 8, convergence_eps: float = 1e-3, s_clip: float = 16.0,
                       s_damping: float = 0.0, original_len: Optional[int] = None, group=None,
                       device: Optional[torch.device] = None, decoder: Optional[Callable] = None,
                       timings: Optional[dict] = None, span: Optional[int] = None):
    """decompress_audio (fractal.py:1378-1473) with the ranges split across the ranks of ``group``.

    ``matches_soa`` ({idx, s, o, sym} arrays) and ``domains`` ([n_domains, range_size] f32) are read on rank 0 only.
    Returns on rank 0 ``(recon numpy f32, info)`` with info = {iterations, deltas, blocks}; None elsewhere.
    ``decoder`` (tests) builds the rank-local decoder; the default is :class:`ShardDecoder` on the rank's GPU, whose
    shard bounds must sit on multiples of ``fwav_decode_span()`` (``span`` overrides it for a test decoder)."""
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    tm = timings if timings is not None else {}
    t0 = time.perf_counter()
    meta = torch.zeros(3, dtype=torch.int64, device=device)
    if rank == 0:
        meta[0], meta[1], meta[2] = int(n_ranges), int(np.asarray(domains).shape[0]), int(range_size)
    _broadcast_(meta, group, device)
    nr, nd, rs = (int(v) for v in meta.cpu().tolist())
    if decoder is None and rs > RESIDENT_MAX_RS:
        # the sharded kernels keep a range in registers (fwav_decode_run: range_size ≤ 32, tile ≤ 8447); longer
        # ranges decode on rank 0 alone with the single-device streaming path — every rank learnt rs from the one
        # broadcast above, so all of them leave here together, before any other collective
        if rank != 0:
            return None
        from . import engine
        td = lambda a, t: torch.from_numpy(np.ascontiguousarray(a, dtype=t)).to(device)  # noqa: E731
        rec, ran, deltas = engine.decompress_device(
            td(matches_soa["idx"], np.int32), td(matches_soa["s"], np.float32), td(matches_soa["o"], np.float32),
            td(np.asarray(matches_soa["sym"]).astype(np.uint8), np.uint8),
            td(np.asarray(domains).reshape(-1), np.float32), nr, rs, iterations, convergence_eps, s_clip, s_damping)
        out = rec.cpu().numpy()
        if original_len is not None:
            out = out[:original_len]
        tm.update(decode_s=time.perf_counter() - t0)
        return out, dict(iterations=ran, deltas=deltas, blocks=[(0, nr)] + [(nr, nr)] * (world - 1))
    pool = torch.empty(max(nd * rs, 1), dtype=torch.float32, device=device)
    if rank == 0 and nd:
        pool[:nd * rs].copy_(torch.from_numpy(np.ascontiguousarray(domains, dtype=np.float32).reshape(-1)))
    _broadcast_(pool, group, device)
    bounds = decode_bounds(nr, world, span)
    maxlen = max(1, max(b - a for a, b in bounds))
    cd = _coll_device(group, device)
    mine = torch.empty((4, maxlen), dtype=torch.int32, device=cd)
    slist = None
    if rank == 0:
        idx = np.asarray(matches_soa["idx"], np.int32)
        s = np.asarray(matches_soa["s"], np.float32)
        o = np.asarray(matches_soa["o"], np.float32)
        sym = np.asarray(matches_soa["sym"]).astype(np.int32)
        slist = []
        for a, b in bounds:
            p = np.zeros((4, maxlen), np.int32)
            p[0, :b - a] = idx[a:b]
            p[1, :b - a] = s[a:b].view(np.int32)
            p[2, :b - a] = o[a:b].view(np.int32)
            p[3, :b - a] = sym[a:b]
            slist.append(torch.from_numpy(p).to(cd))
    dist.scatter(mine, scatter_list=slist, src=0, group=group)
    lo, hi = bounds[rank]
    m = hi - lo
    mine = mine.to(device)
    idx_l = mine[0, :m].contiguous()
    s_l = mine[1, :m].contiguous().view(torch.float32)
    o_l = mine[2, :m].contiguous().view(torch.float32)
    sym_l = mine[3, :m].to(torch.uint8)
    _sync(device)
    t1 = time.perf_counter()
    make = decoder or ShardDecoder
    dec = make(idx_l, s_l, o_l, sym_l, pool[:max(nd * rs, 1)], lo, nr, rs, iterations, convergence_eps, s_clip,
               s_damping)
    rec, ran, deltas = decode_shard(dec, group, device)
    _sync(device)
    t2 = time.perf_counter()
    buf = torch.zeros(maxlen * rs, dtype=torch.float32, device=cd)
    buf[:m * rs] = rec[:m * rs].to(cd)
    glist = [torch.empty_like(buf) for _ in range(world)] if rank == 0 else None
    dist.gather(buf, gather_list=glist, dst=0, group=group)
    _sync(device)
    t3 = time.perf_counter()
    tm.update(distribute_s=t1 - t0, decode_s=t2 - t1, gather_s=t3 - t2)
    if rank != 0:
        return None
    out = torch.cat([glist[r][:(b - a) * rs] for r, (a, b) in enumerate(bounds)]).cpu().numpy()
    if original_len is not None:
        out = out[:original_len]
    return out, dict(iterations=ran, deltas=deltas, blocks=bounds)
