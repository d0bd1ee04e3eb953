"""Candidate rows at full-size tables against the oracle: the product's rows compared,
order included, with O.topk_rows — the reference's sgemv order for the process's OpenBLAS thread count (above
nd = 28,800 numpy splits `domain_embs @ q`, fractal.py:537, over its threads) and numpy's own argpartition/argsort
(fractal.py:538-541) on every row with an exact tie among its top K + 1 — and each match tuple with O.affine of the
ORACLE's candidate row (fractal.py:757-850).  Test helper, not a test module."""
from __future__ import annotations

import numpy as np

from oracle import fractal_oracle as O


def row_scores(emb: np.ndarray, q: np.ndarray, cand_row: np.ndarray, threads: int) -> np.ndarray:
    """Reference-order scores of the domains cand_row (−1 → NaN)."""
    c = np.asarray(cand_row, np.int64)
    ok = c >= 0
    out = np.full(len(c), np.nan, np.float32)
    if ok.any():
        out[ok] = O.sgemv_scores(emb[c[ok]], q[None, :], O.sgemv_col_kind(c[ok], len(emb), threads))[0]
    return out


def check_rows(emb: np.ndarray, pool: np.ndarray, ranges: np.ndarray, cand: np.ndarray, outs, rows, k: int,
               threads: int, q_offset: int = 0, exact=(), chunk: int = 64, label: str = "") -> dict:
    """``rows``: local indices of unpruned ranges (into cand / ranges / outs, queries emb[q_offset + row]).
    * a row whose oracle top K + 1 holds no exact tie (and every row of ``exact``: rows the product re-ranked with
      numpy's own calls) equals the oracle's row, order included;
    * a row with an exact tie that the product left in (score desc, index asc) order — its tie check found that
      numpy's order cannot change the match — holds the same reference-order score at every position, and the same
      domain at every position whose score is unique in the top K + 1;
    * every match tuple (idx, s, o, sym, err) equals O.affine of the oracle's candidate row, bit for bit.
    Returns counts (rows, near-gap rows with K-th − (K+1)-th < 1e-5, tied rows, tied rows left in device order)."""
    rows = np.asarray(rows, np.int64)
    oc, kth, k1th, tied = O.topk_rows(emb, q_offset + rows, k, threads, chunk=chunk,
                                      row_scores=lambda q: O.reference_row_scores(emb, q, threads))
    got = cand[rows]
    exact = set(int(r) for r in exact)
    gap = (kth.astype(np.float64) - k1th.astype(np.float64))
    near = int(np.sum(np.nan_to_num(gap, nan=1.0) < 1e-5))
    loose = 0
    for j, r in enumerate(rows):
        if not tied[j] or int(r) in exact:
            assert np.array_equal(got[j], oc[j]), (label, int(r), got[j], oc[j])
            continue
        if np.array_equal(got[j], oc[j]):
            continue
        loose += 1
        q = emb[q_offset + r]
        a = row_scores(emb, q, got[j], threads)
        b = row_scores(emb, q, oc[j], threads)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), (label, int(r))
        vals = np.append(b, k1th[j])
        uniq = np.array([np.sum(vals == v) == 1 for v in b])
        assert np.array_equal(got[j][uniq], oc[j][uniq]), (label, int(r))
    want = O.affine(ranges[rows], oc, pool)
    for nm, t, v in zip(("idx", "s", "o", "sym", "err"), outs, want):
        t = np.asarray(t)[rows]
        assert np.array_equal(t.view(np.uint8), np.asarray(v).view(np.uint8)), (label, nm)
    out = dict(rows=len(rows), near_gap=near, tied=int(tied.sum()), tied_device_order=loose)
    print(f"{label}: {out}")
    return out
