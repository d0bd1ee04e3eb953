"""Match records: the reference's ``list[(domain_idx, s, o, sym, err)]`` backed by SoA arrays.

``compress_audio`` returns one Python tuple per range (fractal.py:837-850, 1240-1245); building 21.6 M
tuples at cfg4 would dominate the GPU path, so :class:`MatchList` keeps the five arrays and materialises a
tuple — with the reference's Python types ``(int, float, float, int, float)`` — only when indexed.
``save_compressed`` / ``decompress_audio`` read the arrays directly; plain lists of tuples are accepted
everywhere too.
"""
from __future__ import annotations

from collections.abc import Sequence

import numpy as np

MATCH_DTYPE = np.dtype([("idx", "<i4"), ("s", "<f4"), ("o", "<f4"), ("sym", "u1"), ("err", "<f4")])  # '<iffBf'


class MatchList(Sequence):
    __slots__ = ("idx", "s", "o", "sym", "err")

    def __init__(self, idx, s, o, sym, err):
        self.idx = np.asarray(idx, np.int32)
        self.s = np.asarray(s, np.float32)
        self.o = np.asarray(o, np.float32)
        self.sym = np.asarray(sym, np.uint8)
        self.err = np.asarray(err, np.float32)

    def __len__(self):
        return len(self.idx)

    def __getitem__(self, i):
        if isinstance(i, slice):
            return [self[j] for j in range(*i.indices(len(self)))]
        return (int(self.idx[i]), float(self.s[i]), float(self.o[i]), int(self.sym[i]), float(self.err[i]))

    def __iter__(self):
        return iter(zip(self.idx.tolist(), self.s.tolist(), self.o.tolist(), self.sym.tolist(), self.err.tolist()))

    def __eq__(self, other):
        try:
            return len(self) == len(other) and all(a == b for a, b in zip(self, other))
        except TypeError:
            return NotImplemented

    def __repr__(self):
        return f"MatchList(n={len(self)})"

    def tolist(self):
        return list(self)


def as_match_arrays(matches):
    """(idx i32, s f32, o f32, sym u8, err f32) from a MatchList or any sequence of 5-tuples."""
    if isinstance(matches, MatchList):
        return matches.idx, matches.s, matches.o, matches.sym, matches.err
    n = len(matches)
    if n == 0:
        return (np.zeros(0, np.int32), np.zeros(0, np.float32), np.zeros(0, np.float32), np.zeros(0, np.uint8),
                np.zeros(0, np.float32))
    idx = np.fromiter((int(m[0]) for m in matches), np.int64, n)
    s = np.fromiter((float(m[1]) for m in matches), np.float64, n)
    o = np.fromiter((float(m[2]) for m in matches), np.float64, n)
    sym = np.fromiter((int(m[3]) for m in matches), np.int64, n)
    err = np.fromiter((float(m[4]) for m in matches), np.float64, n)
    return idx.astype(np.int32), s.astype(np.float32), o.astype(np.float32), sym.astype(np.uint8), err.astype(np.float32)
