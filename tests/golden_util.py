"""Golden fixture access + the SURVEY Appendix A parity rules (test helpers)."""
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


def candidate_agreement(cand, gold_cand, kth, k1th, emb_q, pruned, gap=1e-5):
    """Rule 3: candidate SETS equal except where the golden K-th/(K+1)-th gap <= 1e-5 (or, when emb_q is given, the
    query is all zero; pass None now that zero queries reproduce the reference's order, quirk Q11).
    Returns (same_set bool[nr], unexplained bool[nr])."""
    same = np.array([set(a.tolist()) == set(b.tolist()) for a, b in zip(cand, gold_cand)])
    zeroq = np.all(emb_q == 0, axis=1) if emb_q is not None else np.zeros(len(cand), bool)
    near = (kth - k1th) <= gap
    unexplained = ~same & ~zeroq & ~near & ~pruned
    return same, unexplained


def match_agreement(idx, sym, err, g, K, cand=None, gap=1e-5, rel=1e-5):
    """Appendix A rule 4 for the end-to-end tuples of golden case g at K: every range whose (domain_index,
    symmetry_flag) differs from the reference's must fit equally well (reference-formula error within `rel`
    relative of the golden error, both +inf for pruned ranges) or be explained by rule 3 (its golden K-th/(K+1)-th
    score gap <= `gap`, so the candidate sets may legitimately differ).  Returns (exact bool[nr], equal_fit
    bool[nr], near bool[nr], unexplained bool[nr])."""
    gi, gs, ge = g[f"m_idx_{K}"], g[f"m_sym_{K}"], g[f"m_err_{K}"]
    idx, sym, err = np.asarray(idx), np.asarray(sym), np.asarray(err, np.float64)
    exact = (idx == gi) & (sym == gs)
    ge64 = ge.astype(np.float64)
    with np.errstate(invalid="ignore", divide="ignore"):
        r = np.abs(err - ge64) / np.maximum(np.abs(ge64), 1e-30)
    equal_fit = (r <= rel) | (np.isinf(err) & np.isinf(ge64))
    kth, k1 = g[f"kth_{K}"], g[f"k1th_{K}"]
    near = (kth - k1) <= gap
    unexplained = ~exact & ~equal_fit & ~near
    return exact, equal_fit, near, unexplained


#: (idx, sym) agreement with the reference measured for the oracle (same scores and tie order as the HIP kernels) —
#: the floors the parity tests hold; the remaining mismatches are equal fits (identical tiles) or exact-tie
#: candidate sets.
MATCH_FLOOR = {("tone", 32): 0.20, ("sweep", 32): 0.999, ("sweep", 64): 1.0, ("noise2048", 64): 1.0,
               ("noise4096", 64): 1.0, ("speech4096", 64): 0.993, ("ragged", 16): 1.0, ("ragged", 2000): 1.0,
               ("tiny", 8): 1.0}

#: scores are bit-identical to the reference's (sgemv order), so candidate sets may differ only where the golden K-th
#: and (K+1)-th scores are exactly equal (numpy's introselect then chooses among the tied domains)
EXACT_TIE_GAP = 0.0
#: the HIP path scores with its OWN embeddings, which are within 1.5e-7 of the reference's (Appendix A rule 2, not
#: bit-exact), so its scores may differ from the reference's by a few 1e-7 and near-ties at the K-th place may flip:
#: the GPU tests apply rule 3's 1e-5 gap (given the same embeddings the kernels equal the oracle exactly:
#: tools/diag/sweep_cands.py)
GPU_TIE_GAP = 1e-5
#: (idx, sym) agreement floors for the HIP path (its own embeddings): measured rates, rounded down
GPU_MATCH_FLOOR = {**MATCH_FLOOR, ("sweep", 32): 0.998, ("sweep", 64): 0.999, ("speech4096", 64): 0.99}
