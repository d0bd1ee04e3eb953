"""The reference's Python API on the MI355X engine (drop-in for ``fractal.py``'s codec functions).

Signatures, defaults, return tuples and error cases follow ``/root/reference/fractal.py``:
  compress_audio      :1045-1273     decompress_audio :1378-1473     compute_snr :1478-1487
  process_file_compress :1491-1521   process_file_decompress :1524-1546

Documented deviations:
  * ``use_gpu`` is accepted and ignored — the hot path always runs on the HIP device (no CPU fallback).
  * ``top_k``: the reference ignores the keyword and always uses the module global ``fractal.top_k`` (= 32,
    quirk Q2).  Here an explicit ``top_k=`` is honoured; when omitted, the module global is used, so calls that
    do not pass it behave exactly like the reference.
  * ``batch_size=`` (what the reference's own test_e2e.py passes) is accepted as an alias of ``batch_size_cpu``;
    the batch sizes, ``ef_search``, ``domains_tmpdir``, ``transient_weight``, ``n_mels`` and ``cpu_workers``
    only shape the reference's process pipeline / unused helpers and do not change results.
  * ``matches`` is a :class:`~fwav.matches.MatchList` (a sequence of the same tuples, array-backed).
  * ``decompress_audio`` returns a host numpy array (the reference returns a CuPy array on its GPU path).
"""
from __future__ import annotations

import logging
import os
import time

import numpy as np
import torch

from . import engine
from .fwavio import load_compressed, read_wav_mono, save_compressed, write_wav
from .matches import MatchList, as_match_arrays

logger = logging.getLogger("fwavc")

#: module-level K, as the reference's ``top_k = 32`` (fractal.py:77)
top_k = 32
EMBED_K = 32
FWAV_VERSION = 1


def _default_k():
    import sys
    mod = sys.modules.get("fractal")
    k = getattr(mod, "top_k", None) if mod is not None else None
    return int(k) if k is not None else int(top_k)


def compress_audio(signal, framerate, sampwidth, tile_size=1024, emb_dim=16, top_k=None, ef_search=50, use_gpu=False,
                   energy_thresh=1e-4, domains_tmpdir=None, batch_size_gpu=512, batch_size_cpu=128, fast_mode=True,
                   transient_weight=1.0, n_mels=40, cpu_workers=None, batch_size=None, device=None):
    """fractal.py:1045 — returns ``(matches, domains, n_ranges, range_size, tile_size, domain_step,
    energy_thresh, original_len)``."""
    if emb_dim != 16:
        raise NotImplementedError("the MI355X engine implements the reference's default emb_dim=16 only")
    k = _default_k() if top_k is None else int(top_k)
    dev = engine.require_device(device)
    sig = np.asarray(signal, dtype=np.float32)
    rs, step = engine.geometry(tile_size)
    t = torch.from_numpy(np.ascontiguousarray(sig)).to(dev)
    copy = _PoolCopy(dev)
    res = engine.compress_device(t, tile_size, k, energy_thresh=energy_thresh, fast_mode=fast_mode,
                                 on_pool=copy.start)
    return device_result_to_tuple(res, copy)


_side_streams: dict = {}


class _PoolCopy:
    """Device→host copy of the domain pool on a side stream, started as soon as the pool kernel is queued so that it
    overlaps the similarity search (the pool is the largest host output: nd × rs f32).  The destination is pinned
    (torch's caching host allocator reuses it across calls) and is handed to the caller as a numpy view."""

    def __init__(self, dev: torch.device):
        self.dev, self.host, self.done = dev, None, None

    def start(self, pool: torch.Tensor) -> None:
        side = _side_streams.get(self.dev)
        if side is None:
            side = _side_streams[self.dev] = torch.cuda.Stream(self.dev)
        ready = torch.cuda.Event()
        ready.record(torch.cuda.current_stream(self.dev))
        self.host = torch.empty(pool.numel(), dtype=pool.dtype, pin_memory=True)
        with torch.cuda.stream(side):
            side.wait_event(ready)
            self.host.copy_(pool, non_blocking=True)
            pool.record_stream(side)
            self.done = torch.cuda.Event()
            self.done.record(side)

    def result(self) -> np.ndarray:
        self.done.synchronize()
        return self.host.numpy()


def device_result_to_tuple(res: "engine.DeviceCompressed", pool_copy: "_PoolCopy | None" = None):
    rs, tile, step, thr, orig = res.range_size, res.tile_size, res.domain_step, res.energy_thresh, res.original_len
    empty = ([], np.zeros((0, rs), dtype=np.float32), 0, rs, tile, step, thr, orig)
    if res.empty or res.is_silent():
        return empty
    # the five match arrays into pinned buffers, one synchronisation for all of them
    src = (res.idx, res.s, res.o, res.sym, res.err)
    hs = [torch.empty(t.numel(), dtype=t.dtype, pin_memory=True) for t in src]
    for h, t in zip(hs, src):
        h.copy_(t, non_blocking=True)
    torch.cuda.current_stream(res.idx.device).synchronize()
    matches = MatchList(*[h.numpy() for h in hs])
    if pool_copy is not None and pool_copy.done is not None:
        domains = pool_copy.result().reshape(res.n_domains, rs)
    else:
        domains = res.pool.view(res.n_domains, rs).cpu().numpy()
    return (matches, domains, res.n_ranges, rs, tile, step, thr, orig)


def decompress_audio(matches, domains_array, n_ranges, range_size, iterations=8, convergence_eps=1e-3, use_gpu=False,
                     original_len=None, s_clip=16.0, s_damping=0.0, device=None, return_info=False):
    """fractal.py:1378 — reconstruct; output trimmed to ``original_len`` when given."""
    dev = engine.require_device(device)
    idx, s, o, sym, _ = as_match_arrays(matches)
    nr, rs = int(n_ranges), int(range_size)
    if len(idx) != nr:
        raise ValueError(f"len(matches)={len(idx)} != n_ranges={nr}")
    dom = np.ascontiguousarray(np.asarray(domains_array, dtype=np.float32))
    if nr > 0 and (dom.size == 0 or dom.shape[-1] != rs):
        raise ValueError("domains_array must be (n_domains, range_size)")
    if nr > 0 and (idx.max(initial=-1) >= len(dom)):
        raise IndexError("domain index out of range")
    td = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    pool = td(dom.reshape(-1)) if dom.size else torch.zeros(max(rs, 1), dtype=torch.float32, device=dev)
    recon, ran, deltas = engine.decompress_device(td(idx), td(s), td(o), td(sym), pool, nr, rs, iterations,
                                                  convergence_eps, s_clip, s_damping)
    for i, d in enumerate(deltas):
        logger.debug(f"Iteration {i + 1}: delta={d:.6e}")
    if deltas and deltas[-1] < convergence_eps:
        logger.info(f"Converged after {ran} iterations (delta={deltas[-1]:.3e})")
    out = recon.cpu().numpy()
    if original_len is not None:
        out = out[:original_len]
    if return_info:
        return out, dict(iterations=ran, deltas=deltas)
    return out


def compute_snr(original, reconstructed):
    """fractal.py:1478-1487."""
    n = min(len(original), len(reconstructed))
    orig = np.asarray(original[:n], dtype=np.float64)
    recon = np.asarray(reconstructed[:n], dtype=np.float64)
    noise = orig - recon
    signal_power = np.sum(orig * orig)
    noise_power = np.sum(noise * noise)
    if noise_power <= 0:
        return float("inf")
    return 10.0 * np.log10(signal_power / noise_power)


def process_file_compress(path, outdir=None, tile=1024, energy_thresh=1e-4, use_gpu=False):
    """fractal.py:1491-1521 (the positional CLI OUTPUT is used as a directory, quirk Q8)."""
    try:
        start = time.time()
        signal, framerate, sampwidth = read_wav_mono(path)
        if sampwidth == 4:
            signal = np.clip(signal.astype(np.float32), -1.0, 1.0)
        matches, domains, n_ranges, range_size, tile_size, domain_step, energy_threshold, original_len = \
            compress_audio(signal, framerate, sampwidth, tile_size=tile, energy_thresh=energy_thresh, use_gpu=use_gpu)
        logger.info(f"Processed {len(matches)} ranges, domain matrix shape {domains.shape}")
        if outdir and not os.path.exists(outdir):
            os.makedirs(outdir)
        outpath = (os.path.splitext(path)[0] + ".fwav") if outdir is None else \
            os.path.join(outdir, os.path.basename(path) + ".fwav")
        save_compressed(outpath, matches, domains, range_size, framerate, sampwidth, tile_size, domain_step,
                        energy_threshold, original_len)
        elapsed = time.time() - start
        in_size = os.path.getsize(path)
        out_size = os.path.getsize(outpath)
        ratio = in_size / out_size if out_size > 0 else 0
        logger.info(f"Compressed {path} -> {outpath}  time={elapsed:.2f}s  ratio={ratio:.2f}")
        return {"input": path, "output": outpath, "time_s": elapsed, "ratio": ratio}
    except Exception as e:  # noqa: BLE001 — the reference returns an error dict, never raises
        logger.exception("Compression failed for %s", path)
        return {"input": path, "error": str(e)}


def process_file_decompress(path, outdir=None, iterations=8, eps=1e-3, use_gpu=False):
    """fractal.py:1524-1546."""
    try:
        start = time.time()
        (matches, domains, n_ranges, range_size, framerate, sampwidth, tile_size, domain_step, energy_threshold,
         original_len) = load_compressed(path)
        recon = decompress_audio(matches, domains, n_ranges, range_size, iterations=iterations, convergence_eps=eps,
                                 use_gpu=use_gpu, original_len=original_len)
        if outdir and not os.path.exists(outdir):
            os.makedirs(outdir)
        if sampwidth == 4:
            recon = np.clip(recon, -1.0, 1.0)
        outpath = (os.path.splitext(path)[0] + "_recon.wav") if outdir is None else \
            os.path.join(outdir, os.path.basename(path) + "_recon.wav")
        write_wav(outpath, np.asarray(recon), framerate, sampwidth)
        elapsed = time.time() - start
        logger.info(f"Decompressed {path} -> {outpath}  time={elapsed:.2f}s")
        return {"input": path, "output": outpath, "time_s": elapsed}
    except Exception as e:  # noqa: BLE001
        logger.exception("Decompression failed for %s", path)
        return {"input": path, "error": str(e)}
