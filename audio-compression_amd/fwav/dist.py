"""Multi-GPU compress: ranges of ONE signal sharded across ranks (one process per GPU, torch.distributed).

Exchange pattern:
  1. rank 0 holds the signal; ONE broadcast of the raw signal (f32, 4 B/sample: 691 MB at cfg4) over
     RCCL/xGMI.  Broadcasting the signal instead of the domain pool (2.76 GB at cfg4) is cheaper and
     sufficient: every rank rebuilds voiced mask, ranges, pool and embeddings bit-identically in a few ms,
     whereas the pool alone would not give the ranges (they need the signal and the voiced-state scan over
     the whole signal).
  2. each rank searches + solves a contiguous block of ranges, blocks balanced by the number of ranges
     that survive the energy prune (silent stretches cost nothing);
  3. the SoA match arrays (17 B/range) are all-gathered into rank 0's result.
No collective runs inside the search itself.  The per-rank compute is pluggable (``compute``) so the
communication code is exercised on CPU with the gloo backend in tests; the product default is
:func:`fwav.engine.compress_device` on the rank's GPU.
"""
from __future__ import annotations

from typing import Callable, Optional

import numpy as np
import torch
import torch.distributed as dist

from .engine import geometry

FIELDS = ("idx", "s", "o", "sym", "err")


def balanced_bounds(weights: np.ndarray, world: int) -> list[tuple[int, int]]:
    """Contiguous blocks of len(weights) items with ~equal total weight (every item weight >= a floor so
    all-zero stretches still split evenly)."""
    n = len(weights)
    w = np.asarray(weights, np.float64) + 1e-3
    cs = np.concatenate([[0.0], np.cumsum(w)])
    cuts = [0] + [int(np.searchsorted(cs, cs[-1] * r / world, side="left")) for r in range(1, world)] + [n]
    cuts = np.maximum.accumulate(np.clip(cuts, 0, n))
    return [(int(cuts[r]), int(cuts[r + 1])) for r in range(world)]


def approx_active_weights(sig: torch.Tensor, range_size: int, energy_thresh: float) -> np.ndarray:
    """Scheduling heuristic only (the exact prune runs inside each rank's compute): 1 for ranges whose raw
    mean energy clears the prune threshold, else 0."""
    n = sig.numel()
    nr = -(-n // range_size)
    x = torch.zeros(nr * range_size, dtype=torch.float32, device=sig.device)
    x[:n] = sig
    e = (x.view(nr, range_size).double() ** 2).mean(dim=1)
    return (e >= 0.75 * energy_thresh).cpu().numpy().astype(np.float64)


def _pack(fields: dict, length: int, device) -> torch.Tensor:
    out = torch.zeros((5, length), dtype=torch.int32, device=device)
    m = len(fields["idx"])
    out[0, :m] = fields["idx"].to(torch.int32)
    out[1, :m] = fields["s"].view(torch.int32)
    out[2, :m] = fields["o"].view(torch.int32)
    out[3, :m] = fields["sym"].to(torch.int32)
    out[4, :m] = fields["err"].view(torch.int32)
    return out


def _device_compute(sig, tile_size, top_k, energy_thresh, shard):
    from .engine import compress_device
    r = compress_device(sig, tile_size, top_k, energy_thresh=energy_thresh, shard=shard)
    if r.empty:
        return None
    return dict(idx=r.idx, s=r.s, o=r.o, sym=r.sym, err=r.err, pool=r.pool, n_ranges=r.n_ranges,
                n_domains=r.n_domains, silent=r.is_silent)


def compress_sharded(signal: Optional[np.ndarray], tile_size: int, top_k: int, energy_thresh: float = 1e-4,
                     group=None, device: Optional[torch.device] = None,
                     compute: Optional[Callable] = None):
    """Compress one signal with its ranges split across the ranks of ``group``.

    ``signal`` is read on rank 0 only (other ranks may pass None).  Returns, on rank 0, a dict with the
    full SoA match arrays (numpy), ``pool`` (numpy [n_domains, range_size]), n_ranges, range_size,
    domain_step, original_len, and the per-rank blocks; other ranks return None.
    """
    rank = dist.get_rank(group)
    world = dist.get_world_size(group)
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    compute = compute or _device_compute
    n_t = torch.zeros(1, dtype=torch.int64, device=device)
    if rank == 0:
        n_t[0] = int(len(signal))
    dist.broadcast(n_t, src=0, group=group)
    n = int(n_t.item())
    sig = torch.empty(n, dtype=torch.float32, device=device)
    if rank == 0:
        sig.copy_(torch.from_numpy(np.ascontiguousarray(signal, dtype=np.float32)))
    dist.broadcast(sig, src=0, group=group)  # the one data-path collective before the search

    rs, step = geometry(tile_size)
    nr = -(-n // rs)
    blocks = balanced_bounds(approx_active_weights(sig, rs, energy_thresh), world)
    lo, hi = blocks[rank]
    res = compute(sig, tile_size, top_k, energy_thresh, (lo, hi))
    maxlen = max(b - a for a, b in blocks)
    if res is None:  # empty / short / silent input: identical decision on every rank
        return dict(empty=True, n_ranges=0, range_size=rs, domain_step=step, original_len=n) if rank == 0 else None
    mine = _pack(res, max(maxlen, 1), device)
    allp = torch.empty((world * 5, max(maxlen, 1)), dtype=torch.int32, device=device)
    dist.all_gather_into_tensor(allp, mine, group=group)
    allp = allp.view(world, 5, -1)
    if rank != 0:
        return None
    allp = allp.cpu()
    parts = {f: [] for f in FIELDS}
    for r, (a, b) in enumerate(blocks):
        m = b - a
        parts["idx"].append(allp[r, 0, :m].numpy().astype(np.int32))
        parts["s"].append(allp[r, 1, :m].numpy().view(np.float32))
        parts["o"].append(allp[r, 2, :m].numpy().view(np.float32))
        parts["sym"].append(allp[r, 3, :m].numpy().astype(np.uint8))
        parts["err"].append(allp[r, 4, :m].numpy().view(np.float32))
    out = {f: np.concatenate(v) for f, v in parts.items()}
    pool = res["pool"]
    pool = pool.cpu().numpy() if isinstance(pool, torch.Tensor) else np.asarray(pool)
    out.update(empty=bool(res["silent"]()) if callable(res.get("silent")) else False, n_ranges=nr, range_size=rs,
               domain_step=step, original_len=n, pool=pool.reshape(-1, rs), blocks=blocks)
    return out
