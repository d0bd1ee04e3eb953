"""ctypes binding of ``libfwav.so`` — the C-ABI boundary declared in ``include/fwav.h``.

The product path has no CPU fallback: if the library (built by ``__graft_entry__.build()``) is missing or
no HIP device is visible, every entry point raises :class:`FwavError`.
"""
from __future__ import annotations

import ctypes as C
import os
import sys

from . import _digest

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libfwav.so")
DEBUG_LIB_PATH = os.path.join(_HERE, "libfwav_debug.so")

P = C.c_void_p
I64 = C.c_int64
I32 = C.c_int
F32 = C.c_float
F64 = C.c_double
SZ = C.c_size_t

#: name → (restype, argtypes); must match include/fwav.h exactly (tests/test_capi.py checks the header).
SIGNATURES = {
    "fwav_last_error": (C.c_char_p, []),
    "fwav_abi_version": (I32, []),
    "fwav_build_digest": (C.c_char_p, []),
    "fwav_stream_sync": (I32, [P]),
    "fwav_voiced_workspace_size": (SZ, [I64, I32]),
    "fwav_voiced_ranges": (I32, [P, I64, I32, I32, I32, F32, F32, P, I64, P, P, SZ, P]),
    "fwav_debug_smooth": (I32, [P, I64, I32, P, P]),
    "fwav_weighted_energy_workspace_size": (SZ, [I64]),
    "fwav_weighted_energy": (I32, [P, I64, P, P, SZ, P]),
    "fwav_prune": (I32, [P, I64, I64, I32, F32, I32, P, I64, I32, P, P, P, P, P]),
    "fwav_emb16_elems": (SZ, [I64]),
    "fwav_embed_tables_size": (SZ, [I32]),
    "fwav_embed_tables": (I32, [I32, P]),
    "fwav_debug_dct2": (I32, [I32, I32, P, P]),
    "fwav_pool_workspace_size": (SZ, [I64, I32, I32, I32]),
    "fwav_pool_embed": (I32, [P, I64, I32, I32, I32, P, P, P, P, P, SZ, P]),
    "fwav_topk_max_k": (I32, []),
    "fwav_sim_topk_workspace_size": (SZ, [I64, I64, I32]),
    "fwav_sim_topk": (I32, [P, P, I64, P, P, I64, I64, I32, I32, P, P, P, SZ, P]),
    "fwav_score_rows": (I32, [P, I64, P, I64, I64, I32, P, P]),
    "fwav_debug_gather_rows": (I32, [P, I64, I32, I64, P, P]),
    "fwav_affine": (I32, [P, I64, I32, P, I32, P, I64, F32, P, P, P, P, P, P]),
    "fwav_tie_check": (I32, [P, I64, I32, P, I32, P, I64, P, I64, I32, P, I64, I32, P, P]),
    "fwav_tie_rows_in": (I32, [P, I64, P, I32, P, P, I32, P, P]),
    "fwav_tie_rows_out": (I32, [P, I64, P, P, P, P, P, P, P, P, P, P, P]),
    "fwav_tie_list_size": (I64, [I64]),
    "fwav_emb16_from_emb": (I32, [P, I64, P, P]),
    "fwav_decode_workspace_size": (SZ, [I64, I32, I32]),
    "fwav_decode": (I32, [P, P, P, P, I64, I32, P, I64, I32, F64, F32, F64, P, P, P, P, P, SZ, P]),
    "fwav_decode_span": (I32, []),
    "fwav_decode_chunk_iterations": (I32, []),
    "fwav_decode_n_chunks": (I32, [I32, F64]),
    "fwav_decode_partials_count": (SZ, [I64]),
    "fwav_decode_from": (I32, [P, P, P, P, I64, I32, P, I64, I32, F64, F32, F64, P, P, P, P, P, P, SZ, P]),
    "fwav_decode_exact": (I32, [P, P, I64, F64, I32, P, P, P]),
    "fwav_decode_all_workspace_size": (SZ, [I64, I32, I32]),
    "fwav_decode_all": (I32, [P, P, P, P, I64, I32, P, I64, I32, F64, F32, F64, P, P, P, P, P, SZ, P]),
    "fwav_decode_run": (I32, [P, P, P, P, I64, I64, I64, I32, P, I64, I32, I32, F64, F32, F64, P, P, P, P, P, P]),
    "fwav_decode_reduce": (I32, [P, I64, I32, I32, I32, F64, P, P, P]),
    "fwav_decode_finish": (I32, [P, P, P, P, I64, I64, I64, I32, P, I64, I32, F64, F32, F64, P, P, P, P, P]),
}

#: the debug library's extra entry points (include/fwav_debug.h): the search's process-global test knobs and
#: diagnostics; libfwav.so exports none of them
DEBUG_SIGNATURES = {
    "fwav_debug_sim_topk": (I32, [P, P, I64, P, P, I64, I64, I32, P, P, SZ, I32, P, P]),
    "fwav_debug_topk_plan": (I32, [I32, I32]),
    "fwav_debug_topk_tail": (I32, [I32]),
    "fwav_debug_topk_plan_cover": (I32, [I64, I32, I32, I32, P, P]),
    "fwav_debug_topk_mode": (I32, [I32]),
    "fwav_debug_topk_geometry": (I32, [I32]),
    "fwav_debug_topk_plan_info": (I32, [I64, I64, P, P]),
    "fwav_debug_topk_piece_chunks": (I32, [I64, I64, I64, P, P]),
    "fwav_debug_topk_qb": (I64, [I32]),
    "fwav_debug_topk_floor": (I32, [I32, F32]),
    "fwav_debug_topk_floor_pieces": (I32, [I32]),
    "fwav_debug_sim_topk_layout": (I32, [I64, I64, P]),
}


class FwavError(RuntimeError):
    """A C-ABI call returned a non-zero status (message from ``fwav_last_error``)."""


_libs: dict = {}
_active = None  # the debug library inside debug_library(), else the product library


#: set by fwav.hipctypes, the torch-free host: the library then binds the system HIP runtime on its own
TORCH_FREE = False


def _one_runtime() -> None:
    """One HIP runtime per process.  PyTorch-ROCm ships its own libamdhip64 (same soname, libamdhip64.so.7, but
    torch's libraries ask for it by another name), so a process that loads libfwav.so — which binds the system
    runtime — before torch ends up with two HIP runtimes, and the second one to initialise sees no device
    ("no ROCm-capable device is detected").  Loaded after torch, libfwav.so binds torch's runtime.  So unless the
    caller is torch-free, torch is imported first."""
    if TORCH_FREE or "torch" in sys.modules:
        return
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def _load(path: str, sigs: dict) -> C.CDLL:
    _one_runtime()
    if not os.path.exists(path):
        raise FwavError(f"HIP library not built: {path} is missing (run __graft_entry__.build())")
    dll = C.CDLL(path)
    dll.fwav_build_digest.restype = C.c_char_p
    built = dll.fwav_build_digest().decode()
    want = _digest.source_digest()
    if want is not None and built != want:
        raise FwavError(f"{path} was built from other sources (digest {built[:12]}, sources {want[:12]}): "
                        "run __graft_entry__.build()")
    for name, (res, args) in sigs.items():
        fn = getattr(dll, name)
        fn.restype = res
        fn.argtypes = args
    return dll


def product_lib() -> C.CDLL:
    """libfwav.so, the product library (include/fwav.h)."""
    if "product" not in _libs:
        _libs["product"] = _load(LIB_PATH, SIGNATURES)
    return _libs["product"]


def debug_lib() -> C.CDLL:
    """libfwav_debug.so (include/fwav_debug.h): the same entry points plus the search's test knobs; tests only.
    FWAV_DEBUG_TOPK_FLOOR="mode[:value]" / FWAV_DEBUG_TOPK_GEOMETRY=g set fwav_debug_topk_floor / _geometry when it
    loads (same-box A/Bs of whole programs, e.g. bench.py under FWAV_DEBUG_LIBRARY=1)."""
    if "debug" not in _libs:
        _libs["debug"] = _load(DEBUG_LIB_PATH, {**SIGNATURES, **DEBUG_SIGNATURES})
        fl = os.environ.get("FWAV_DEBUG_TOPK_FLOOR")
        if fl:
            mode, _, value = fl.partition(":")
            _libs["debug"].fwav_debug_topk_floor(int(mode), float(value or 0.0))
        if os.environ.get("FWAV_DEBUG_TOPK_GEOMETRY"):
            _libs["debug"].fwav_debug_topk_geometry(int(os.environ["FWAV_DEBUG_TOPK_GEOMETRY"]))
        if os.environ.get("FWAV_DEBUG_TOPK_TAIL"):
            _libs["debug"].fwav_debug_topk_tail(int(os.environ["FWAV_DEBUG_TOPK_TAIL"]))
        if os.environ.get("FWAV_DEBUG_TOPK_P2"):
            _libs["debug"].fwav_debug_topk_floor_pieces(int(os.environ["FWAV_DEBUG_TOPK_P2"]))
    return _libs["debug"]


def lib() -> C.CDLL:
    """The library every fwav call goes through: the product library, or the debug one inside debug_library() (or
    for the whole process under FWAV_DEBUG_LIBRARY=1: the experiment scripts in tools/ set it)."""
    if _active is not None:
        return _active
    return debug_lib() if os.environ.get("FWAV_DEBUG_LIBRARY") == "1" else product_lib()


class debug_library:
    """``with debug_library(): ...`` routes every fwav call of the block (fwav.engine included) through
    libfwav_debug.so, whose process-global knobs (fwav_debug_topk_plan / _mode / _geometry / _floor) the block may set; they
    are reset to the defaults on exit.  Test-only: not thread-safe, not re-entrant across threads."""

    def __enter__(self):
        global _active
        self.prev = _active
        _active = debug_lib()
        return _active

    def __exit__(self, *exc):
        global _active
        d = debug_lib()
        d.fwav_debug_topk_plan(-1, 1)
        d.fwav_debug_topk_mode(-1)
        d.fwav_debug_topk_geometry(-1)
        d.fwav_debug_topk_floor(-1, 0.0)
        d.fwav_debug_topk_floor_pieces(0)
        d.fwav_debug_topk_tail(-1)
        _active = self.prev
        return False


def call(name: str, *args) -> int:
    L = lib()
    rc = getattr(L, name)(*args)
    if rc != 0:
        msg = L.fwav_last_error().decode(errors="replace")
        raise FwavError(f"{name} failed ({rc}): {msg}")
    return rc


def size_call(name: str, *args) -> int:
    return int(getattr(lib(), name)(*args))


#: fwav_debug_sim_topk_layout's regions, in its order
SIM_TOPK_LAYOUT = ("keys", "share", "ovf2", "n_ovf2", "seeds2", "ovf1", "n_ovf1", "seeds1", "miss", "n_miss", "miss2",
                   "n_miss2", "floor_key", "order", "n_order", "order_bits", "order_bsum", "pilot", "total")


def sim_topk_layout(max_q: int, n_domains: int) -> dict:
    """Byte offsets of the fp16 search's workspace regions (the debug library's fwav_debug_sim_topk_layout; every
    region before ``pilot`` sits at the same offset in libfwav.so).  Tests and diagnostics read the tail through this,
    never by arithmetic of their own."""
    out = (C.c_int64 * len(SIM_TOPK_LAYOUT))()
    rc = debug_lib().fwav_debug_sim_topk_layout(int(max_q), int(n_domains), out)
    if rc != 0:
        raise FwavError(f"fwav_debug_sim_topk_layout: {rc}")
    return dict(zip(SIM_TOPK_LAYOUT, (int(v) for v in out)))
