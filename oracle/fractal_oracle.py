"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement (numpy / scipy) of the reference hot path, ``/root/reference/fractal.py``.
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this module,
and only as the checker / the timed CPU baseline: the product path (``audio-compression_amd/fwav``) never
imports it and fails loudly when its HIP library is missing.

Pinning: every function below is checked against the golden vectors in ``tests/golden/*.npz``, which
``tests/golden/make_golden.py`` produced by running the reference's own functions in this container
(tests/test_oracle_golden.py).  Bit-exact where the reference's float32 arithmetic is reproducible
(pool, ranges, voiced mask, affine, decode, .fwav bytes); within SURVEY.md Appendix A tolerances where it
is not (embeddings: pocketfft + BLAS-dot norms; candidate sets: BLAS sgemv order).

Arithmetic spec:
  * every reduction along the last axis uses numpy's ``pairwise_sum`` order, including numpy's initial
    ``0 +`` (so a sum of −0.0 values is +0.0);  ``mean = sum / float32(n)``;
  * every elementwise op is one separately rounded float32 op (no FMA);
  * Python-float constants meeting float32 arrays are rounded to float32 first (NEP 50).
"""
from __future__ import annotations

import hashlib
import struct

import numpy as np
import scipy.fftpack

F32 = np.float32
FWAV_VERSION = 1          # fractal.py:59
HEADER_FMT = "<4sBIIBHHfIII"   # fractal.py:1291-1301
HEADER_SIZE = struct.calcsize(HEADER_FMT)  # 34
MATCH_DTYPE = np.dtype([("idx", "<i4"), ("s", "<f4"), ("o", "<f4"), ("sym", "u1"), ("err", "<f4")])  # '<iffBf'


# ----------------------------------------------------------------------------------------- reductions
def _pw(x: np.ndarray) -> np.ndarray:
    """numpy pairwise_sum (loops_utils.h.src) along the last axis, vectorised over leading axes."""
    n = x.shape[-1]
    if n < 8:
        r = np.zeros(x.shape[:-1], F32)
        for i in range(n):
            r = r + x[..., i]
        return r
    if n <= 128:
        m = n - n % 8
        blk = x[..., :m].reshape(x.shape[:-1] + (m // 8, 8))
        r = blk[..., 0, :].copy()
        for i in range(1, m // 8):
            r = r + blk[..., i, :]
        res = ((r[..., 0] + r[..., 1]) + (r[..., 2] + r[..., 3])) + ((r[..., 4] + r[..., 5]) + (r[..., 6] + r[..., 7]))
        for i in range(m, n):
            res = res + x[..., i]
        return res
    n2 = n // 2
    n2 -= n2 % 8
    return _pw(x[..., :n2]) + _pw(x[..., n2:])


def pw_sum(x: np.ndarray) -> np.ndarray:
    """``np.add.reduce(x, axis=-1)`` for float32, order made explicit (initial value 0, then pairwise)."""
    x = np.asarray(x, F32)
    return F32(0.0) + _pw(x)


def pw_mean(x: np.ndarray) -> np.ndarray:
    return pw_sum(x) / F32(x.shape[-1])


def sdot_f32(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """Short BLAS sdot, as np.linalg.norm of a 1-D float32 vector evaluates it (fractal.py:205 ``sqrt(e.dot(e))``):
    OpenBLAS's x86_64 sdot runs n < 32 entirely in its tail loop, ``double dot += (float)(y[i] * x[i])`` — each
    product rounded to float32, accumulated in float64 in index order, the sum rounded to float32 on return.
    Measured bit-exact against numpy (OpenBLAS 0.3.29) on every golden embedding row; rows batched."""
    acc = np.zeros(a.shape[:-1], np.float64)
    for i in range(a.shape[-1]):
        acc = acc + (a[..., i] * b[..., i]).astype(np.float64)
    return acc.astype(F32)


def seq_dot_f64(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    acc = np.zeros(a.shape[:-1], np.float64)
    for i in range(a.shape[-1]):
        acc = acc + a[..., i] * b[..., i]
    return acc


# ------------------------------------------------------------------------------- geometry / constants
def geometry(tile_size: int):
    """range_size / domain_step (fractal.py:1070-1071)."""
    rs = max(4, tile_size // 256)
    return rs, max(1, rs // 4)


def prune_threshold(energy_thresh: float) -> np.float32:
    """``np.mean(r**2) < energy_thresh * 0.75`` compares float32 vs a weak Python float (fractal.py:602)."""
    return F32(energy_thresh * 0.75)


# ------------------------------------------------------------------------------------- voiced (a6)
def frame_energies(signal: np.ndarray, frame_size: int) -> np.ndarray:
    """fractal.py:885-891: reflect-pad to whole frames, float32 pairwise mean of squares per frame."""
    signal = np.asarray(signal, F32)
    n = len(signal)
    n_frames = (n + frame_size - 1) // frame_size
    pad = n_frames * frame_size - n
    padded = np.pad(signal, (0, pad), mode="reflect") if pad else signal
    frames = padded.reshape(n_frames, frame_size)
    return pw_mean(frames * frames)


def smooth5(e: np.ndarray, smooth_window: int = 5) -> np.ndarray:
    """``np.convolve(e, ones(w,f32)/w, 'same')`` (fractal.py:893-895) as numpy evaluates it, measured against
    np.convolve on wide-range random energies (tests/test_oracle_golden.py::test_smooth_matches_numpy):
      n ≥ w: output i covers e[i − w//2 : i − w//2 + w] ∩ [0, n).  A full window is numpy's small_correlate: f32
             products added in f32, in e order.  A partial window (the first w//2 and last w − w//2 − 1 outputs) is
             the dtype dot (OpenBLAS sdot): f32 products accumulated in float64 in e order, then rounded.
      n < w: numpy swaps the operands (correlate of the kernel with reversed e) and returns w outputs; output j covers
             the e indices i with 0 ≤ t − i ≤ w − 1, t = j + (n − 1)//2.  A full overlap (all n) is f32 in reversed e
             order, a partial one the float64-accumulated dot in reversed e order."""
    w = smooth_window
    k = F32(1.0) / F32(w)  # np.ones(w, f32) / w  → float32
    e = np.asarray(e, F32)
    n = len(e)

    def f32_seq(idx):
        s = F32(0.0)
        for i in idx:
            s = F32(s + F32(e[i] * k))
        return s

    def f64_dot(idx):
        s = 0.0
        for i in idx:
            s += float(F32(e[i] * k))
        return F32(s)

    if n < w:
        out = np.empty(w, F32)
        off = (n - 1) // 2
        for j in range(w):
            t = j + off
            idx = [i for i in range(n - 1, -1, -1) if 0 <= t - i <= w - 1]
            out[j] = f32_seq(idx) if len(idx) == n else f64_dot(idx)
        return out
    left = w // 2
    out = np.empty(n, F32)
    # full windows, vectorised (same f32 order as the scalar loop)
    mid = n - w + 1
    acc = np.zeros(mid, F32)
    for j in range(w):
        acc = acc + e[j:j + mid] * k
    out[left:left + mid] = acc
    for i in list(range(left)) + list(range(left + mid, n)):
        lo, hi = max(0, i - left), min(n, i - left + w)
        out[i] = f64_dot(range(lo, hi))
    return out


def hysteresis(e: np.ndarray, hi: float, lo: float) -> np.ndarray:
    """fractal.py:900-907 (sequential scan) vectorised: a frame's state is the decision of the last frame
    that was > hi (voiced) or < lo (unvoiced); comparisons in float32 (NEP 50)."""
    hi32, lo32 = F32(hi), F32(lo)
    dec = np.where(e > hi32, 1, np.where(e < lo32, 0, -1))
    pos = np.where(dec >= 0, np.arange(len(e)), -1)
    last = np.maximum.accumulate(pos) if len(pos) else pos
    return np.where(last >= 0, dec[np.maximum(last, 0)], 0).astype(np.uint8)


def voiced_detection(signal, frame_size=64, energy_threshold=1e-4, smooth_window=5, low_threshold=None):
    """fractal.py:880-909."""
    signal = np.asarray(signal, F32)
    n = len(signal)
    e = frame_energies(signal, frame_size)
    if smooth_window > 1:
        e = smooth5(e, smooth_window)
    if low_threshold is None:
        low_threshold = energy_threshold * 0.5
    vm = hysteresis(e, energy_threshold, low_threshold)
    return np.repeat(vm, frame_size)[:n]


def form_ranges(signal: np.ndarray, mask: np.ndarray, rs: int):
    """fractal.py:1079-1112 → (ranges f32[nr, rs], original_len)."""
    ws = np.asarray(signal, F32) * mask
    orig = len(ws)
    pad = (rs - orig % rs) % rs
    if pad:
        ws = np.pad(ws, (0, pad), mode="reflect")
    return ws.reshape(-1, rs), orig


# ------------------------------------------------------------------------------- domain pool (a1)
def domain_pool(signal: np.ndarray, tile: int, rs: int, step: int, block: int = 2048) -> np.ndarray:
    """build_domains_memmap (fractal.py:285-334): pool[d, k] = pairwise-mean(signal[d*step + k*bl : +bl])."""
    signal = np.asarray(signal, F32)
    n = len(signal)
    if n < tile:
        return np.zeros((0, rs), F32)
    win = np.lib.stride_tricks.sliding_window_view(signal, tile)[::step]
    nd = win.shape[0]
    bl = tile // rs
    out = np.empty((nd, rs), F32)
    for i in range(0, nd, block):
        b = win[i:i + block, :bl * rs].reshape(-1, rs, bl)
        out[i:i + len(b)] = pw_mean(b)
    return out


# ---------------------------------------------------------------------------------- embedding (a2)
def embed(pool: np.ndarray, emb_dim: int = 16) -> np.ndarray:
    """build_domain_embeddings → multi_head_embedding (fractal.py:166-208, 154-164), rows batched.
    Tonal head: float32 ortho DCT-II (scipy.fftpack, as the reference), × linspace(1,2,n) (f64), drop DC,
    first ≤k coefficients → f32, zero-pad, L2-normalise (f32) if norm > 1e-8.
    Transient head: diff(prepend=x0) (f32) × linspace (f64) → f64 ortho DCT-II → first ≤k → normalise (f64)."""
    pool = np.asarray(pool, F32)
    nd, n = pool.shape
    tk = emb_dim // 2
    out = np.zeros((nd, emb_dim), F32)
    if nd == 0:
        return out
    w = np.linspace(1.0, 2.0, n)
    v = scipy.fftpack.dct(pool, norm="ortho", axis=-1) * w
    take = min(tk, max(0, n - 1))
    e = np.zeros((nd, tk), F32)
    e[:, :take] = v[:, 1:1 + take].astype(F32)
    nrm = np.sqrt(sdot_f32(e, e))
    ok = nrm > F32(1e-8)
    e[ok] = e[ok] / nrm[ok, None]
    d = np.diff(pool, axis=-1, prepend=pool[:, :1]) * w
    t = scipy.fftpack.dct(d, norm="ortho", axis=-1)[:, :tk]
    tn = np.sqrt(seq_dot_f64(t, t))
    okt = tn > 1e-8
    t[okt] = t[okt] / tn[okt, None]
    out[:, :tk] = e
    out[:, tk:tk + t.shape[1]] = t.astype(F32)
    return out


# ------------------------------------------------------------------------------- candidates (a4)
def range_energy_pruned(ranges: np.ndarray, energy_thresh: float, fast_mode: bool = True) -> np.ndarray:
    if not fast_mode:
        return np.zeros(len(ranges), bool)
    return pw_mean(ranges * ranges) < prune_threshold(energy_thresh)


def numpy_topk_row(scores: np.ndarray, k: int) -> np.ndarray:
    """range_candidates_from_embedding_emb (fractal.py:535-541) + pad_candidates (:544-552) on one score row, by the
    same numpy calls: argpartition(scores, −K)[−K:] ordered by argsort(...)[::-1] (a full argsort when K ≥ nd), −1
    padded to K.  Exactly equal scores come out in the order numpy's selection and sort leave them."""
    nd = len(scores)
    if k >= nd:
        idx = np.argsort(scores)[::-1]
    else:
        part = np.argpartition(scores, -k)[-k:]
        idx = part[np.argsort(scores[part])[::-1]]
    out = np.full(k, -1, np.int32)
    out[:min(k, len(idx))] = idx[:k]
    return out


def zero_query_candidates(nd: int, k: int) -> np.ndarray:
    """The row of an all-zero query (quirk Q11): every score is 0, so numpy's tie order decides the whole row."""
    return numpy_topk_row(np.zeros(nd, F32), k)


def blas_threads() -> int:
    """OpenBLAS's thread count in this process (what numpy's sgemv would split over; sgemv_col_kind), read from the
    OpenBLAS numpy bundles (its get_num_threads).  Raises when it cannot be read — never a guess."""
    import ctypes
    import glob
    import os
    root = os.path.dirname(os.path.dirname(np.__file__))
    libs = sorted(glob.glob(os.path.join(root, "numpy.libs", "*openblas*")))
    if not libs:
        import threadpoolctl
        libs = sorted({i["filepath"] for i in threadpoolctl.threadpool_info() if i.get("internal_api") == "openblas"})
    got = []
    for path in libs:
        h = ctypes.CDLL(path)
        for sym in ("scipy_openblas_get_num_threads64_", "scipy_openblas_get_num_threads",
                    "openblas_get_num_threads64_", "openblas_get_num_threads"):
            if hasattr(h, sym):
                got.append(int(getattr(h, sym)()))
                break
    if len(got) != 1 or got[0] < 1:
        raise RuntimeError(f"cannot read numpy's OpenBLAS thread count from {libs}")
    return got[0]


#: OpenBLAS (interface/gemv.c) runs sgemv single-threaded while m·n < 115200·GEMM_MULTITHREAD_THRESHOLD (= 4)
SGEMV_THREAD_MIN_MN = 460_800


def sgemv_col_kind(cols, nd: int, threads: int) -> np.ndarray:
    """Which OpenBLAS sgemv_t kernel scores column (domain) d of the reference's ``domain_embs @ q`` (fractal.py:537):
    0 = the 4-column microkernel, 1 = the 4x2 tail kernel, 2 = the 4x1 tail kernel.  gemv_thread.c splits the nd
    columns over T threads (T = 1 while 16·nd < SGEMV_THREAD_MIN_MN, else OpenBLAS's thread count) in widths
    ceil(rest / threads left) — the first nd mod T chunks one column wider — and each thread's sgemv_t scores its
    chunk's last (width mod 4) columns with the tail kernels (2 → 4x2, 1 → 4x1, 3 → 4x2 then 4x1).  Pinned against
    numpy here for T = 1, 3, 5, 7, 8 and nd from 577 to 6.6 M (every column bit-exact)."""
    d = np.asarray(cols, np.int64)
    T = 1 if 16 * nd < SGEMV_THREAD_MIN_MN else max(1, int(threads))
    q, r = divmod(int(nd), T)
    big = d < r * (q + 1)
    w = np.where(big, q + 1, q)
    start = np.where(big, d // (q + 1) * (q + 1), r * (q + 1) + (d - r * (q + 1)) // max(q, 1) * q)
    pos = d - start
    t = w & 3
    body = pos < w - t
    two = ((t & 2) != 0) & (pos < w - t + 2)
    return np.where(body, 0, np.where(two, 1, 2)).astype(np.int8)


def sgemv_scores(emb: np.ndarray, q: np.ndarray, kinds=None) -> np.ndarray:
    """emb @ q for a block of queries q (R, 16), in the order the reference's BLAS evaluates it (fractal.py:537:
    numpy sgemv → OpenBLAS 0.3.29 sgemv_t, Haswell/SkylakeX kernels), per column kind (sgemv_col_kind; None = all 0):
      0: 8 fma lanes l_j = fma(d[j+8], q[j+8], 0 + d[j]·q[j]), then ((l0 + l4) + (l1 + l5)) + ((l2 + l6) + (l3 + l7));
      1: 4 SSE lanes l_j = ((0 + p_j) + p_{j+4}) + p_{j+8}) + p_{j+12} of rounded products p, then (l0 + l1) + (l2 + l3);
      2: 8 lanes l_j = (0 + p_j) + p_{j+8}, then ((l0 + l4) + (l1 + l5)) + ((l2 + l6) + (l3 + l7)).
    Bit-exact against numpy on every column (sgemv_col_kind).  Returns (R, n) float32."""
    E = np.asarray(emb, F32)
    Q = np.asarray(q, F32)
    P = [Q[:, None, j] * E[None, :, j] for j in range(16)]          # rounded f32 products
    z = F32(0)
    lanes = []
    for j in range(8):
        p = Q[:, None, j + 8].astype(np.float64) * E[None, :, j + 8].astype(np.float64)  # exact
        lanes.append(fma_f32(p, (z + P[j]).astype(np.float64)))
    r = [lanes[i] + lanes[i + 4] for i in range(4)]
    out = (r[0] + r[1]) + (r[2] + r[3])
    if kinds is None or not np.any(kinds):
        return out
    kinds = np.asarray(kinds)
    l4 = [(((z + P[j]) + P[j + 4]) + P[j + 8]) + P[j + 12] for j in range(4)]
    a = (l4[0] + l4[1]) + (l4[2] + l4[3])
    l8 = [(z + P[j]) + P[j + 8] for j in range(8)]
    r8 = [l8[i] + l8[i + 4] for i in range(4)]
    b = (r8[0] + r8[1]) + (r8[2] + r8[3])
    return np.where(kinds[None, :] == 1, a, np.where(kinds[None, :] == 2, b, out))


def fma_f32(p: np.ndarray, c: np.ndarray) -> np.ndarray:
    """round_to_f32(p + c) for an exact f64 product p of two f32 and an f32 value c, i.e. f32 fma: s = fl64(p + c)
    with its exact error e (TwoSum); fl32(s) is the correctly rounded result unless s lies exactly on a midpoint of
    two f32 neighbours (s is the nearest f64 to p + c, and f32 midpoints are f64 values), where the sign of e
    decides instead of ties-to-even."""
    s = p + c
    bb = s - p
    e = (p - (s - bb)) + (c - bb)
    r = s.astype(F32)
    r64 = r.astype(np.float64)
    other = np.nextafter(r, np.where(s > r64, np.float32(np.inf), np.float32(-np.inf)).astype(F32))
    mid = (r64 + other.astype(np.float64)) * 0.5
    fix = (s == mid) & (e != 0)
    if fix.any():
        hi = np.maximum(r, other)
        lo = np.minimum(r, other)
        r = np.where(fix, np.where(e > 0, hi, lo), r)
    return r


#: bound on the difference between two f32 summation orders of a 16-term dot product whose Σ|q_k d_k| ≤ 2 (each is
#: within 15·2^-24·2 ≈ 1.8e-6 of the exact value), with margin
SGEMV_GAP = 8e-6


def reference_row_scores(emb: np.ndarray, q: np.ndarray, threads: int, chunk: int = 1 << 23) -> np.ndarray:
    """One whole score row ``domain_embs @ q`` (fractal.py:537) in the reference's order.  When ``threads`` is this
    process's OpenBLAS thread count, numpy's own call IS the reference's computation (the restatement below is pinned
    bit for bit against it: tests/test_oracle_golden.py::test_sgemv_thread_split_pinned_against_numpy), and takes
    0.1 s instead of 4 s for a 6.6 M-domain row; otherwise the restatement, in column chunks (bounded memory)."""
    E = np.asarray(emb, F32)
    q = np.asarray(q, F32)
    nd = len(E)
    if int(threads) == blas_threads():
        return E @ q
    out = np.empty(nd, F32)
    for a in range(0, nd, chunk):
        cols = np.arange(a, min(nd, a + chunk))
        out[a:a + len(cols)] = sgemv_scores(E[a:a + len(cols)], q[None, :], sgemv_col_kind(cols, nd, threads))[0]
    return out


def topk_rows(emb: np.ndarray, qrows, k: int, threads: int, chunk: int = 512, row_scores=None):
    """The reference's candidate rows (fractal.py:535-552) for the queries emb[qrows] (quirk Q1: query i is domain row
    i), none of them pruned.  Rows whose top K + 1 scores are all distinct are decided by the scores alone (score
    desc; the K-th beats the (K+1)-th); a row with exactly equal scores among its top K + 1 — and every all-zero query
    (quirk Q11) — is scored in full and handed to numpy's own argpartition/argsort (numpy_topk_row), whose tie order
    the reference inherits.  ``row_scores(q)``: the whole reference-order score row of query vector q (default: the
    restatement for ``threads``; reference_row_scores).  Returns (cand i32[n, k] −1-padded, kth f32[n], k1th f32[n],
    tied bool[n]: an exact tie among the top K + 1 — every all-zero query counts as tied)."""
    E = np.asarray(emb, F32)
    nd = E.shape[0]
    qrows = np.asarray(qrows, np.int64)
    n = len(qrows)
    cand = np.full((n, k), -1, np.int32)
    kth = np.full(n, np.nan, F32)
    k1th = np.full(n, np.nan, F32)
    tied = np.zeros(n, bool)
    kk = min(k, nd)
    zero = np.all(E[qrows] == 0, axis=1) if n else np.zeros(0, bool)
    if zero.any():
        cand[zero] = zero_query_candidates(nd, k)
        kth[zero] = 0
        k1th[zero] = 0
        tied[zero] = True
    act = np.nonzero(~zero)[0]
    kind_all = None
    for s in range(0, len(act), chunk):
        pos = act[s:s + chunk]
        # BLAS scores (another summation order: within SGEMV_GAP of the sgemv order) pick a superset of every
        # domain that can be in the exact top K + 1; the superset is then scored in the sgemv order and selected exactly
        fast = E[qrows[pos]] @ E.T
        if kk < nd:
            # the (K+1)-th BLAS score — of every stride-th column on large tables: a subset's (K+1)-th is at most the
            # whole row's, so the superset below still holds the exact top K + 1 (a few hundred columns wider)
            stride = max(1, nd // (1 << 20))
            sub = fast[:, ::stride] if stride > 1 else fast
            Tf = -np.partition(-sub, kk, axis=1)[:, kk] if sub.shape[1] > kk else sub.min(axis=1)
            del sub
        else:
            Tf = fast.min(axis=1)
        for j, p in enumerate(pos):
            q = E[qrows[p]]
            sup = np.nonzero(fast[j] >= Tf[j] - SGEMV_GAP)[0]
            ex = sgemv_scores(E[sup], q[None, :], sgemv_col_kind(sup, nd, threads))[0]
            o = np.lexsort((sup, -ex))  # (score desc, index asc)
            top = ex[o[:kk + 1]]
            if np.any(top[1:] == top[:-1]):
                tied[p] = True
                if row_scores is not None:
                    full = row_scores(q)
                else:
                    if kind_all is None:
                        kind_all = sgemv_col_kind(np.arange(nd), nd, threads)
                    full = sgemv_scores(E, q[None, :], kind_all)[0]
                cand[p] = numpy_topk_row(full, k)
            else:
                cand[p, :kk] = sup[o[:kk]]
            kth[p] = ex[o[kk - 1]]
            if kk < nd:
                k1th[p] = ex[o[kk]]
        del fast
    return cand, kth, k1th, tied


def topk_candidates(emb: np.ndarray, n_ranges: int, k: int, pruned: np.ndarray, chunk: int = 512,
                    threads: int | None = None, stats: dict | None = None, rows=None, row_scores=None):
    """cpu_worker + range_candidates_from_embedding_emb + pad_candidates (fractal.py:556-632, 535-552): the energy
    prune (pruned rows stay all −1, :602) and topk_rows for every other range — or only for ``rows``.  Scores in
    float32 in the reference's sgemv order for ``threads`` OpenBLAS threads (default: this process's).  Returns
    (cand i32[nr, k] −1-padded, kth f32[nr], k1th f32[nr]); stats['ties'] counts the rows with an exact tie in
    their top K + 1 (all-zero queries aside) and stats['tie_rows'] lists them."""
    nd = emb.shape[0]
    threads = blas_threads() if threads is None else int(threads)
    cand = np.full((n_ranges, k), -1, np.int32)
    kth = np.full(n_ranges, np.nan, F32)
    k1th = np.full(n_ranges, np.nan, F32)
    want = np.zeros(n_ranges, bool)
    if rows is None:
        want[:] = True
    else:
        want[np.asarray(rows, np.int64)] = True
    act = np.nonzero(want & ~pruned[:n_ranges])[0]
    c, a, b, tied = topk_rows(emb, act, k, threads, chunk=chunk, row_scores=row_scores)
    cand[act], kth[act], k1th[act] = c, a, b
    if stats is not None:
        zero = np.all(np.asarray(emb)[act] == 0, axis=1) if len(act) else np.zeros(0, bool)
        stats["tie_rows"] = act[tied & ~zero].tolist()
        stats["ties"] = len(stats["tie_rows"])
    return cand, kth, k1th


def topk_candidates_loop(emb: np.ndarray, rows: np.ndarray, k: int) -> np.ndarray:
    """Per-range sgemv + argpartition, the reference's cost structure (fractal.py:537-541) — CPU baseline."""
    out = np.empty((len(rows), k), np.int32)
    nd = emb.shape[0]
    for j, i in enumerate(rows):
        scores = emb @ emb[i]
        if k >= nd:
            idx = np.argsort(scores)[::-1]
        else:
            idx = np.argpartition(scores, -k)[-k:]
            idx = idx[np.argsort(scores[idx])[::-1]]
        out[j, :len(idx)] = idx[:k]
    return out


# ----------------------------------------------------------------------------------- affine (a5)
def affine(ranges: np.ndarray, cand: np.ndarray, pool: np.ndarray, s_clip: float = 16.0):
    """_process_gpu_batch (fractal.py:757-850), float32 in numpy order.  Returns SoA (idx, s, o, sym, err)."""
    ranges = np.asarray(ranges, F32)
    B, N = ranges.shape
    K = cand.shape[1]
    safe = np.where(cand < 0, 0, cand)
    dom = pool[safe]                                     # (B, K, N)
    dsym = np.concatenate([dom, dom[:, :, ::-1]], axis=1)  # (B, 2K, N) contiguous
    r_mean = pw_mean(ranges)[:, None]                    # (B, 1)
    r_c = ranges - r_mean
    d_mean = pw_mean(dsym)[:, :, None]                   # (B, 2K, 1)
    d_c = dsym - d_mean
    num = pw_sum(d_c * r_c[:, None, :])
    den = pw_sum(d_c * d_c) + F32(1e-12)
    s = num / den
    o = r_mean - s * d_mean[:, :, 0]
    recon = s[:, :, None] * dsym + o[:, :, None]
    diff = recon - ranges[:, None, :]
    err = np.sqrt(pw_sum(diff * diff))
    inval = np.concatenate([cand < 0, cand < 0], axis=1)
    err = np.where(inval, F32(np.inf), err)
    j = np.argmin(err, axis=1)
    ar = np.arange(B)
    c = abs(F32(s_clip))
    return (np.concatenate([safe, safe], axis=1)[ar, j].astype(np.int32),
            np.clip(s[ar, j], -c, c).astype(F32), o[ar, j].astype(F32),
            (j >= K).astype(np.uint8), err[ar, j].astype(F32))


# ----------------------------------------------------------------------------------- decode (a7)
def sdot_blas(x: np.ndarray, y: np.ndarray) -> np.float32:
    """``x.dot(y)`` of two contiguous float32 vectors as numpy evaluates it (numpy → cblas_sdot, OpenBLAS 0.3.29
    ``kernel/x86_64/sdot.c`` + ``sdot_microk_skylakex-2.c``; one thread whatever OpenBLAS's thread count — measured):
    the first n1 = n & −32 entries by the vector kernel — 64 f32 fma accumulators (4 × 16 lanes; lane l of block b
    takes entry 64b + l) over n & −64 entries, each folded to 8 lanes (a_k[j] = acc_k[j] + acc_k[j+8]), one more
    32-entry fma step (4 × 8 lanes) when n1 is an odd multiple of 32, then ((a0 + a1) + a2) + a3, its upper and lower
    four lanes added, two horizontal adds (h0 + h1) + (h2 + h3) — then the n − n1 tail products (rounded to f32) added
    in f64, the sum rounded to f32.  Pinned against numpy: tests/test_oracle_golden.py::test_sdot_blas_pinned."""
    x = np.ascontiguousarray(x, F32).reshape(-1)
    y = np.ascontiguousarray(y, F32).reshape(-1)
    n = len(x)
    n1 = n & -32
    n64 = n1 & -64
    dot = 0.0
    if n1:
        xb = x[:n64].reshape(-1, 64).astype(np.float64)
        yb = y[:n64].reshape(-1, 64).astype(np.float64)
        acc = np.zeros(64, F32)
        for b in range(len(xb)):  # one fma per lane per block, in block order
            acc = fma_f32(xb[b] * yb[b], acc.astype(np.float64))
        a = (acc.reshape(4, 16)[:, :8] + acc.reshape(4, 16)[:, 8:]).astype(F32)  # (4, 8)
        if n1 != n64:
            xt = x[n64:n1].reshape(4, 8).astype(np.float64)
            yt = y[n64:n1].reshape(4, 8).astype(np.float64)
            a = fma_f32(xt * yt, a.astype(np.float64))
        v = ((a[0] + a[1]) + a[2]) + a[3]
        h = v[:4] + v[4:]
        dot = float((h[0] + h[1]) + (h[2] + h[3]))
    for i in range(n1, n):
        dot += float(x[i] * y[i])  # f32 product, f64 accumulation
    return F32(dot)


def reference_delta(recon: np.ndarray, nxt: np.ndarray) -> float:
    """The convergence measure of decompress_audio (fractal.py:1460-1461) by the reference's own numpy calls:
    ``norm(recon_next − recon) / (norm(recon) if norm(recon) > 0 else 1.0)`` on float32 arrays — np.linalg.norm of a
    1-D float32 vector is sqrt(x.dot(x)) (BLAS sdot, sdot_blas), a float32; the quotient is float32, float() of it."""
    r = np.ascontiguousarray(recon, F32).reshape(-1)
    d = np.ascontiguousarray(nxt, F32).reshape(-1) - r
    nr = np.linalg.norm(r)
    denom = nr if nr > 0 else 1.0
    return float(np.linalg.norm(d) / denom)


def decode(idx, s_st, o_st, sym, pool, n_ranges, range_size, iterations=8, convergence_eps=1e-3,
           original_len=None, s_clip=16.0, s_damping=0.0, deltas="f64"):
    """decompress_audio (fractal.py:1378-1473), float32 in numpy order.  The early exit takes the reference's own
    decision: Δ = reference_delta (numpy's BLAS sdot norms, fractal.py:1460-1461) < eps.  Returns (recon f32,
    iterations_run, deltas): deltas="f64" lists Δ in float64 from exact float64 sums of the same float32 values (what the
    device reports), deltas="reference" the reference's own float32-derived values."""
    idx = np.asarray(idx, np.int32).copy()
    s_st = np.asarray(s_st, F32).copy()
    o_st = np.asarray(o_st, F32).copy()
    sym = np.asarray(sym).astype(bool).copy()
    nr, rs = n_ranges, range_size
    inval = idx < 0
    idx[inval] = 0
    tiles = np.asarray(pool, F32)[idx] if nr else np.zeros((0, rs), F32)
    if inval.any():
        tiles[inval] = 0
        s_st[inval] = 0
        o_st[inval] = 0
        sym[inval] = False
    tiles = np.where(sym[:, None], tiles[:, ::-1], tiles)
    mean_d = pw_mean(tiles)
    tc = tiles - mean_d[:, None]
    den = pw_sum(tc * tc)
    valid = den > F32(1e-12)
    recon = np.zeros((nr, rs), F32)
    c = abs(F32(s_clip))
    out_deltas = []
    it_run = 0
    for _ in range(iterations):
        mr = pw_mean(recon)
        rc = recon - mr[:, None]
        num = pw_sum(rc * tc)
        s_opt = np.zeros(nr, F32)
        s_opt[valid] = num[valid] / den[valid]
        if s_damping > 0:
            s_used = F32(1.0 - s_damping) * s_st + F32(s_damping) * s_opt
        else:
            s_used = np.where(valid, s_opt, s_st)
        s_used = np.clip(s_used, -c, c)
        nxt = F32(0.0) + (s_used[:, None] * tiles + o_st[:, None])   # bincount adds into +0.0
        delta = reference_delta(recon, nxt)
        if deltas == "f64":
            rn = float(np.sqrt(np.sum(recon.astype(np.float64) ** 2)))
            dn = float(np.sqrt(np.sum((nxt - recon).astype(np.float64) ** 2)))  # f32 difference, as :1460
            out_deltas.append(dn / (rn if rn > 0 else 1.0))
        else:
            out_deltas.append(delta)
        recon = nxt
        it_run += 1
        if delta < convergence_eps:
            break
    out = recon.reshape(-1)
    if original_len is not None:
        out = out[:original_len]
    return out, it_run, out_deltas


# ----------------------------------------------------------------------------------- .fwav (format)
def fwav_bytes(idx, s, o, sym, err, pool, range_size, framerate, sampwidth, tile_size, domain_step,
               energy_threshold, original_len) -> bytes:
    """save_compressed (fractal.py:1278-1322) as one byte string."""
    m = np.empty(len(idx), MATCH_DTYPE)
    m["idx"], m["s"], m["o"], m["sym"], m["err"] = idx, s, o, sym, err
    body = np.ascontiguousarray(pool, "<f4").tobytes() + m.tobytes()
    hdr = struct.pack(HEADER_FMT, b"FWAV", FWAV_VERSION, range_size, framerate, sampwidth, tile_size,
                      domain_step, energy_threshold, len(idx), len(pool), original_len)
    return hdr + hashlib.sha256(body).digest() + body


# ------------------------------------------------------------------------------------- pipeline
def compress(signal, tile_size, top_k, energy_thresh=1e-4, fast_mode=True, threads=None):
    """compress_audio (fractal.py:1045-1256) without the process pipeline.  Returns a dict of stages."""
    signal = np.asarray(signal, F32)
    rs, step = geometry(tile_size)
    vm = voiced_detection(signal, frame_size=2 * rs, energy_threshold=energy_thresh)
    ranges, orig = form_ranges(signal, vm, rs)
    pool = domain_pool(signal, tile_size, rs, step)
    emb = embed(pool)
    pruned = range_energy_pruned(ranges, energy_thresh, fast_mode)
    cand, kth, k1th = topk_candidates(emb, len(ranges), top_k, pruned, threads=threads)
    idx, s, o, sym, err = affine(ranges, cand, pool)
    return dict(rs=rs, step=step, voiced=vm, ranges=ranges, original_len=orig, pool=pool, emb=emb,
                pruned=pruned, cand=cand, kth=kth, k1th=k1th, idx=idx, s=s, o=o, sym=sym, err=err)
