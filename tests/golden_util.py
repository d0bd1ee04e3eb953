"""Golden fixture access (test helpers)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CASES = ["tone", "sweep", "noise2048", "noise4096", "speech4096", "ragged", "tiny"]


def load(case):
    g = dict(np.load(os.path.join(GOLDEN, f"{case}.npz")))
    g["p"] = json.loads(str(g.pop("params")))
    return g


def bits(a):
    a = np.asarray(a)
    return a.view(np.uint32) if a.dtype == np.float32 else a


def bit_equal(a, b):
    return np.array_equal(bits(np.asarray(a)), bits(np.asarray(b)))


def same_sets(cand, gold):
    """bool[nr]: row i of cand holds the same candidates as row i of gold (order aside)."""
    return np.array([set(a.tolist()) == set(b.tolist()) for a, b in zip(cand, gold)])
