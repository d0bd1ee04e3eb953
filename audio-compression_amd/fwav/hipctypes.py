"""Torch-free host for libfwav.so: HIP device memory through ctypes on libamdhip64.

This is the binding a maintainer of the reference would add to ``fractal.py``: numpy arrays in,
numpy arrays out, libfwav's C ABI in between, nothing from PyTorch (importing this module imports no torch).  The
product host (fwav.engine) uses torch tensors only as device buffers; :func:`compress` and :func:`decompress` drive
the whole device sequence of INTEGRATION.md §2.3 with HIP buffers alone — the cpu_worker / _process_gpu_batch
pipeline of compress_audio (fractal.py:1040-1256, :556-632, :757-870) and decompress_audio (:1378-1473).
"""
from __future__ import annotations

import ctypes as C
import sys

import numpy as np

from . import geometry
from . import _lib
from ._lib import FwavError, call, size_call
from .nporder import blas_threads, numpy_topk_row, zero_query_candidates

# this host never imports torch: unless torch is already there, libfwav.so binds the system HIP runtime (and hip()
# then reuses whichever runtime it bound)
_lib.TORCH_FREE = "torch" not in sys.modules

_HIP = None
H2D, D2H = 1, 2


def _mapped_runtime():
    """Path of the HIP runtime already mapped into this process (/proc/self/maps), if any."""
    try:
        with open("/proc/self/maps") as f:
            paths = sorted({ln.split()[-1] for ln in f if "libamdhip64" in ln and "/" in ln})
    except OSError:
        return None
    return paths[0] if paths else None


def hip():
    """The HIP runtime libfwav.so is bound to: libfwav.so is loaded first (it binds torch's runtime when torch came
    first, else the system one), and that very library — found in /proc/self/maps — serves the buffers here, so a
    process never maps a second runtime through this module."""
    global _HIP
    if _HIP is None:
        _lib.product_lib()
        mapped = _mapped_runtime()
        for p in ([mapped] if mapped else []) + ["libamdhip64.so", "/opt/rocm/lib/libamdhip64.so"]:
            try:
                _HIP = C.CDLL(p)
                break
            except OSError:
                continue
        if _HIP is None:
            raise FwavError("libamdhip64.so not found")
        _HIP.hipMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t]
        _HIP.hipFree.argtypes = [C.c_void_p]
        _HIP.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        _HIP.hipMemset.argtypes = [C.c_void_p, C.c_int, C.c_size_t]
        _HIP.hipDeviceSynchronize.argtypes = []
    return _HIP


def _ck(rc, what):
    if rc != 0:
        raise FwavError(f"{what}: hipError {rc}")


class DeviceBuffer:
    """hipMalloc'd bytes; freed on close()/GC."""

    def __init__(self, nbytes: int):
        self.nbytes = max(int(nbytes), 1)
        self.ptr = C.c_void_p()
        _ck(hip().hipMalloc(C.byref(self.ptr), self.nbytes), "hipMalloc")

    @classmethod
    def from_array(cls, a: np.ndarray) -> "DeviceBuffer":
        a = np.ascontiguousarray(a)
        b = cls(a.nbytes)
        if a.nbytes:
            _ck(hip().hipMemcpy(b.ptr, a.ctypes.data, a.nbytes, H2D), "hipMemcpy H2D")
        return b

    def to_array(self, dtype, count: int) -> np.ndarray:
        out = np.empty(count, dtype=dtype)
        if out.nbytes:
            _ck(hip().hipDeviceSynchronize(), "hipDeviceSynchronize")
            _ck(hip().hipMemcpy(out.ctypes.data, self.ptr, out.nbytes, D2H), "hipMemcpy D2H")
        return out

    @property
    def value(self) -> int:
        return self.ptr.value

    def close(self):
        if self.ptr:
            hip().hipFree(self.ptr)
            self.ptr = C.c_void_p()

    def __del__(self):  # noqa: D105
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


def affine_batch(ranges: np.ndarray, cand: np.ndarray, pool: np.ndarray, s_clip: float = 16.0):
    """_process_gpu_batch (fractal.py:757-850) for a whole batch: ranges f32[B, rs], cand i32[B, K] (−1 padded),
    pool f32[nd, rs] → (idx i32[B], s f32[B], o f32[B], sym u8[B], err f32[B])."""
    ranges = np.ascontiguousarray(ranges, np.float32)
    cand = np.ascontiguousarray(cand, np.int32)
    pool = np.ascontiguousarray(pool, np.float32)
    B, rs = ranges.shape
    K = cand.shape[1]
    nd = pool.shape[0]
    dr, dc, dp = (DeviceBuffer.from_array(x) for x in (ranges, cand, pool))
    outs = [DeviceBuffer(4 * B), DeviceBuffer(4 * B), DeviceBuffer(4 * B), DeviceBuffer(B), DeviceBuffer(4 * B)]
    call("fwav_affine", dr.value, B, rs, dc.value, K, dp.value, nd, float(abs(np.float32(s_clip))),
         *[b.value for b in outs], None)
    call("fwav_stream_sync", None)
    return (outs[0].to_array(np.int32, B), outs[1].to_array(np.float32, B), outs[2].to_array(np.float32, B),
            outs[3].to_array(np.uint8, B), outs[4].to_array(np.float32, B))


def pool_embed(signal: np.ndarray, tile: int, rs: int, step: int):
    """build_domains_memmap + build_domain_embeddings (fractal.py:285-334, 238-280) →
    (pool f32[nd, rs], emb f32[nd, 16])."""
    sig = np.ascontiguousarray(signal, np.float32)
    n = sig.size
    nd = (n - tile) // step + 1
    tab = np.empty(size_call("fwav_embed_tables_size", rs), np.float64)
    call("fwav_embed_tables", rs, tab.ctypes.data)
    ds, dt = DeviceBuffer.from_array(sig), DeviceBuffer.from_array(tab)
    dpool, demb = DeviceBuffer(4 * nd * rs), DeviceBuffer(4 * nd * 16)
    wsn = size_call("fwav_pool_workspace_size", n, tile, rs, step)
    dws = DeviceBuffer(wsn)
    call("fwav_pool_embed", ds.value, n, tile, rs, step, dt.value, dpool.value, demb.value, None, dws.value, wsn,
         None)
    call("fwav_stream_sync", None)
    return dpool.to_array(np.float32, nd * rs).reshape(nd, rs), demb.to_array(np.float32, nd * 16).reshape(nd, 16)


def _i32(buf: DeviceBuffer, count: int) -> np.ndarray:
    return buf.to_array(np.int32, count)


def compress(signal: np.ndarray, tile_size: int, top_k: int, energy_thresh: float = 1e-4, fast_mode: bool = True,
             s_clip: float = 16.0, tie_order: str = "numpy", threads: int | None = None) -> dict | None:
    """compress_audio's device pipeline (fractal.py:1040-1256) with HIP buffers only, on the null stream:

      fwav_voiced_ranges → fwav_weighted_energy (silent test, :1083) → fwav_pool_embed → fwav_prune → fwav_sim_topk
      → fwav_affine → fwav_tie_check, and for the rows it lists fwav_score_rows + numpy's own ranking
      (argpartition/argsort, :535-541) + fwav_tie_rows_in → fwav_affine → fwav_tie_rows_out.

    Returns None where the reference returns its empty tuple (input shorter than a tile, or silent), raises the
    reference's ValueErrors (empty input; more ranges than domains, quirk Q9), else a dict of host arrays: idx, s, o,
    sym, err (the match tuples), pool f32[nd, rs], emb f32[nd, 16], cand i32[nr, K], n_ranges, range_size,
    domain_step, n_domains, n_ties, n_resolved.  ``tie_order`` as fwav.engine.compress_device ("numpy",
    "numpy_sets", "numpy_rows" or "index")."""
    modes = {"numpy": 0, "numpy_sets": 1, "numpy_rows": 2, "index": -1}  # → fwav_tie_check's exact_sets
    if tie_order not in modes:
        raise ValueError("tie_order must be 'numpy', 'numpy_sets', 'numpy_rows' or 'index'")
    sig = np.ascontiguousarray(signal, np.float32).reshape(-1)
    n = sig.size
    if n == 0:
        raise ValueError("a cannot be empty")  # np.convolve on zero frames (fractal.py:895)
    k = int(top_k)
    rs, step = geometry(tile_size)
    frame = 2 * rs
    nr = -(-n // rs)
    nd = 0 if n < tile_size else (n - tile_size) // step + 1
    T = blas_threads() if threads is None else int(threads)
    thr32, lo32 = np.float32(energy_thresh), np.float32(energy_thresh * 0.5)
    d_sig = DeviceBuffer.from_array(sig)
    d_ranges = DeviceBuffer(4 * nr * rs)
    wsv = size_call("fwav_voiced_workspace_size", n, frame)
    d_wsv = DeviceBuffer(wsv)
    call("fwav_voiced_ranges", d_sig.value, n, rs, frame, 5, float(thr32), float(lo32), d_ranges.value, nr, None,
         d_wsv.value, wsv, None)
    wse = size_call("fwav_weighted_energy_workspace_size", n)
    d_wse, d_part = DeviceBuffer(wse), DeviceBuffer(4)
    call("fwav_weighted_energy", d_ranges.value, n, d_part.value, d_wse.value, wse, None)
    silent = np.float32(d_part.to_array(np.float32, 1)[0]) < np.float32(1e-8)
    if n < tile_size or nr > nd:
        if silent or n < tile_size:
            return None
        raise ValueError("mmap length is greater than file size")  # quirk Q9 (fractal.py:1190-1195)
    if silent:
        return None
    tab = np.empty(size_call("fwav_embed_tables_size", rs), np.float64)
    call("fwav_embed_tables", rs, tab.ctypes.data)
    d_tab = DeviceBuffer.from_array(tab)
    d_pool, d_emb = DeviceBuffer(4 * nd * rs), DeviceBuffer(4 * nd * 16)
    d_emb16 = DeviceBuffer(2 * size_call("fwav_emb16_elems", nd))
    wsp = size_call("fwav_pool_workspace_size", n, tile_size, rs, step)
    d_wsp = DeviceBuffer(wsp)
    call("fwav_pool_embed", d_sig.value, n, tile_size, rs, step, d_tab.value, d_pool.value, d_emb.value,
         d_emb16.value, d_wsp.value, wsp, None)
    d_cand, d_active, d_nact = DeviceBuffer(4 * nr * k), DeviceBuffer(4 * nr), DeviceBuffer(4)
    d_zc = DeviceBuffer.from_array(zero_query_candidates(nd, k))
    call("fwav_prune", d_ranges.value, nr, 0, rs, float(np.float32(energy_thresh * 0.75)), int(bool(fast_mode)),
         d_emb.value, nd, k, d_zc.value, d_cand.value, d_active.value, d_nact.value, None)
    wsk = size_call("fwav_sim_topk_workspace_size", nr, nd, k)
    d_wsk = DeviceBuffer(wsk)
    d_ties = DeviceBuffer(4 * size_call("fwav_tie_list_size", nr))
    call("fwav_sim_topk", d_emb.value, d_emb16.value, nd, d_active.value, d_nact.value, nr, 0, k, T, d_cand.value,
         d_ties.value, d_wsk.value, wsk, None)
    outs = [DeviceBuffer(4 * nr), DeviceBuffer(4 * nr), DeviceBuffer(4 * nr), DeviceBuffer(nr), DeviceBuffer(4 * nr)]
    sc = float(abs(np.float32(s_clip)))
    call("fwav_affine", d_ranges.value, nr, rs, d_cand.value, k, d_pool.value, nd, sc, *[b.value for b in outs], None)
    n_ties = n_res = 0
    if tie_order != "index":
        d_res = DeviceBuffer(4 * (nr + 1))
        call("fwav_tie_check", d_ranges.value, nr, rs, d_cand.value, k, d_pool.value, nd, d_emb.value, 0, T,
             d_ties.value, nr, modes[tie_order], d_res.value, None)
        n_ties = int(_i32(d_ties, 1)[0])
        res = _i32(d_res, 1 + nr)
        n_res = int(res[0])
        if n_res:
            rows = np.ascontiguousarray(res[1:1 + n_res])
            d_rows = DeviceBuffer.from_array(rows)
            # one exact score row at a time (nd floats each; the reference's sgemv order), ranked by numpy
            d_sr = DeviceBuffer(4 * nd)
            newc = np.empty((n_res, k), np.int32)
            for j in range(n_res):
                call("fwav_score_rows", d_emb.value, nd, d_rows.value + 4 * j, 1, 0, T, d_sr.value, None)
                newc[j] = numpy_topk_row(d_sr.to_array(np.float32, nd), k)
            d_newc = DeviceBuffer.from_array(newc)
            d_rsub = DeviceBuffer(4 * n_res * rs)
            call("fwav_tie_rows_in", d_rows.value, n_res, d_newc.value, k, d_cand.value, d_ranges.value, rs,
                 d_rsub.value, None)
            tmp = [DeviceBuffer(4 * n_res), DeviceBuffer(4 * n_res), DeviceBuffer(4 * n_res), DeviceBuffer(n_res),
                   DeviceBuffer(4 * n_res)]
            call("fwav_affine", d_rsub.value, n_res, rs, d_newc.value, k, d_pool.value, nd, sc, *[b.value for b in tmp],
                 None)
            call("fwav_tie_rows_out", d_rows.value, n_res, *[b.value for b in tmp], *[b.value for b in outs], None)
    call("fwav_stream_sync", None)
    return dict(idx=_i32(outs[0], nr), s=outs[1].to_array(np.float32, nr), o=outs[2].to_array(np.float32, nr),
                sym=outs[3].to_array(np.uint8, nr), err=outs[4].to_array(np.float32, nr),
                pool=d_pool.to_array(np.float32, nd * rs).reshape(nd, rs),
                emb=d_emb.to_array(np.float32, nd * 16).reshape(nd, 16), cand=_i32(d_cand, nr * k).reshape(nr, k),
                n_ranges=nr, range_size=rs, domain_step=step, n_domains=nd, n_ties=n_ties, n_resolved=n_res)


def decompress(idx: np.ndarray, s: np.ndarray, o: np.ndarray, sym: np.ndarray, pool: np.ndarray, n_ranges: int,
               range_size: int, iterations: int = 8, convergence_eps: float = 1e-3, s_clip: float = 16.0,
               s_damping: float = 0.0, original_len: int | None = None) -> tuple[np.ndarray, int, list]:
    """decompress_audio (fractal.py:1378-1473) through fwav_decode with HIP buffers only: returns (recon f32,
    iterations run, Δ per iteration), recon trimmed to ``original_len`` when given."""
    nr, rs = int(n_ranges), int(range_size)
    pool = np.ascontiguousarray(pool, np.float32)
    nd = pool.size // rs if rs > 0 else 0
    it = int(iterations)
    d = [DeviceBuffer.from_array(np.ascontiguousarray(a, t)) for a, t in
         ((idx, np.int32), (s, np.float32), (o, np.float32), (sym, np.uint8))]
    d_pool = DeviceBuffer.from_array(pool.reshape(-1) if pool.size else np.zeros(max(rs, 1), np.float32))
    d_a, d_b = DeviceBuffer(4 * max(nr * rs, 1)), DeviceBuffer(4 * max(nr * rs, 1))
    d_del = DeviceBuffer.from_array(np.zeros(max(it, 1), np.float64))
    d_state = DeviceBuffer.from_array(np.zeros(4, np.int32))
    wsn = size_call("fwav_decode_workspace_size", nr, rs, it)
    d_ws = DeviceBuffer(max(wsn, 16))
    eps = float(convergence_eps)
    done, d_init = 0, None
    while True:
        call("fwav_decode_from", *[b.value for b in d], nr, rs, d_pool.value, nd, it - done, eps,
             float(abs(np.float32(s_clip))), float(s_damping), None if d_init is None else d_init.value, d_a.value,
             d_b.value, d_del.value + 8 * done, d_state.value, d_ws.value, wsn, None)
        call("fwav_stream_sync", None)
        state = _i32(d_state, 4)
        ran = int(state[1])
        res, other = (d_b, d_a) if int(state[2]) == 1 else (d_a, d_b)
        if int(state[0]) == 2:  # the early-exit check in the reference's own sdot order (fractal.py:1460-1465)
            call("fwav_decode_exact", other.value, res.value, nr * rs, eps, ran - 1, d_del.value + 8 * done,
                 d_state.value, None)
            call("fwav_stream_sync", None)
            if int(_i32(d_state, 1)[0]) == 3 and done + ran < it:  # the reference goes on: resume from here
                if d_init is None:
                    d_init = DeviceBuffer(4 * max(nr * rs, 1))
                _ck(hip().hipMemcpy(d_init.ptr, res.ptr, 4 * nr * rs, 3), "hipMemcpy")  # device to device
                done += ran
                continue
        done += ran
        break
    ran = done
    out = res.to_array(np.float32, nr * rs)
    if original_len is not None:
        out = out[:original_len]
    return out, ran, d_del.to_array(np.float64, max(it, 1))[:ran].tolist()
