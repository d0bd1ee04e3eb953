"""Minimal torch-free host for libfwav.so: HIP device memory through ctypes on libamdhip64.

This is the binding a maintainer of the reference would add to ``fractal.py``: numpy arrays in,
numpy arrays out, libfwav's C ABI in between, nothing from PyTorch.  The product host (fwav.engine) uses torch
tensors only as device buffers; this module shows the ABI does not depend on them.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import FwavError, call, size_call

_HIP = None
H2D, D2H = 1, 2


def hip():
    global _HIP
    if _HIP is None:
        for p in ("libamdhip64.so", "/opt/rocm/lib/libamdhip64.so"):
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
