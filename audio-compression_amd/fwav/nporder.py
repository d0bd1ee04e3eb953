"""The numpy-only half of the tie handling (no torch): the reference's own ranking of one exact score row, its row for
an all-zero query, and the OpenBLAS thread count whose sgemv order the scores follow.  Used by fwav.ties / fwav.engine
and by the torch-free binding fwav.hipctypes.

Reference: range_candidates_from_embedding_emb (fractal.py:535-541), pad_candidates (:544-552), and the scores
``domain_embs @ q`` (:537) that numpy hands to OpenBLAS's sgemv.
"""
from __future__ import annotations

import os

import numpy as np

_BLAS_GET = None

#: get_num_threads entry points of the OpenBLAS builds numpy ships with (scipy-openblas64, scipy-openblas32, plain)
_OPENBLAS_GET = ("scipy_openblas_get_num_threads64_", "scipy_openblas_get_num_threads", "openblas_get_num_threads64_",
                 "openblas_get_num_threads")


def _openblas_libs() -> list:
    """Candidate files of the OpenBLAS that numpy's ``@`` calls: the one numpy's wheel bundles (``numpy.libs``), else
    the OpenBLAS builds threadpoolctl finds loaded in this process."""
    import glob
    root = os.path.dirname(os.path.dirname(np.__file__))
    libs = sorted(glob.glob(os.path.join(root, "numpy.libs", "*openblas*")))
    if libs:
        return libs
    try:
        import threadpoolctl
        return sorted({i["filepath"] for i in threadpoolctl.threadpool_info() if i.get("internal_api") == "openblas"})
    except ImportError:
        return []


def blas_threads() -> int:
    """OpenBLAS's thread count in this process, read from numpy's own OpenBLAS (its ``get_num_threads``) at every
    call — the split of the reference's sgemv (fractal.py:537) that decides which domains its tail kernels score
    (fwav_common.h).  The reference would run here with the same numpy, so its scores follow this count.
    ``FWAV_BLAS_THREADS`` overrides it.  Raises FwavError when the count cannot be read (no guess: a wrong count
    silently changes which columns take the tail kernels' order)."""
    global _BLAS_GET
    env = os.environ.get("FWAV_BLAS_THREADS")
    if env:
        return max(1, int(env))
    if _BLAS_GET is None:
        import ctypes
        libs = _openblas_libs()
        found = []
        for path in libs:
            h = ctypes.CDLL(path)  # already loaded by numpy: the same handle, so the count is numpy's live one
            for sym in _OPENBLAS_GET:
                if hasattr(h, sym):
                    f = getattr(h, sym)
                    f.restype, f.argtypes = ctypes.c_int, []
                    found.append(f)
                    break
        if len(found) != 1:
            from ._lib import FwavError
            raise FwavError(f"cannot read numpy's OpenBLAS thread count ({len(found)} OpenBLAS builds found in {libs});"
                            " set FWAV_BLAS_THREADS to the reference's thread count")
        _BLAS_GET = found[0]
    n = int(_BLAS_GET())
    if n < 1:
        from ._lib import FwavError
        raise FwavError(f"numpy's OpenBLAS reports {n} threads")
    return n


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




_ZERO_CAND: dict = {}


def zero_query_candidates(n_domains: int, top_k: int) -> np.ndarray:
    """The reference's candidate row for a query whose embedding is all zero (quirk Q11): every score is 0, so the row
    is the order in which numpy's introselect (``argpartition``) and ``argsort`` leave equal keys —
    ``range_candidates_from_embedding_emb`` (fractal.py:535-541) evaluated on a zero score vector, padded with −1 by
    ``pad_candidates`` (fractal.py:544-552).  A K-element constant per (n_domains, K), computed once on the host by
    the same numpy calls the reference makes (the tie order is numpy's, so it is taken from numpy)."""
    key = (int(n_domains), int(top_k))
    if key not in _ZERO_CAND:
        _ZERO_CAND[key] = numpy_topk_row(np.zeros(key[0], np.float32), key[1])
    return _ZERO_CAND[key]
