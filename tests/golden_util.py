"""Golden fixture access + the SURVEY Appendix A parity rules (test helpers)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["tone", "sweep", "noise2048", "noise4096", "speech4096", "ragged"]


def load(case):
    g = dict(np.load(os.path.join(GOLDEN, f"{case}.npz")))
    g["p"] = json.loads(str(g.pop("params")))
    return g


def bits(a):
    a = np.asarray(a)
    return a.view(np.uint32) if a.dtype == np.float32 else a


def bit_equal(a, b):
    return np.array_equal(bits(np.asarray(a)), bits(np.asarray(b)))


def candidate_agreement(cand, gold_cand, kth, k1th, emb_q, pruned, gap=1e-5):
    """Rule 3: candidate SETS equal except where the golden K-th/(K+1)-th gap <= 1e-5 or the query is all zero.
    Returns (same_set bool[nr], unexplained bool[nr])."""
    same = np.array([set(a.tolist()) == set(b.tolist()) for a, b in zip(cand, gold_cand)])
    zeroq = np.all(emb_q == 0, axis=1)
    near = (kth - k1th) <= gap
    unexplained = ~same & ~zeroq & ~near & ~pruned
    return same, unexplained
