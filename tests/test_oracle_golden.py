"""Pin the oracle (CPU restatement) against the reference's own outputs (tests/golden, made by
tests/golden/make_golden.py from /root/reference/fractal.py).  Bars: SURVEY.md Appendix A."""
import numpy as np
import pytest

from golden_util import CASES, bit_equal, load
from oracle import fractal_oracle as O


@pytest.mark.parametrize("case", CASES)
def test_voiced_ranges_pool_bitexact(case):
    g = load(case)
    p = g["p"]
    rs, step = O.geometry(p["tile"])
    assert (rs, step) == (p["rs"], p["step"])
    vm = O.voiced_detection(g["signal"], 2 * rs, p["thr"])
    assert np.array_equal(vm, g["voiced"])
    r, orig = O.form_ranges(g["signal"], vm, rs)
    assert orig == p["original_len"]
    assert bit_equal(r, g["ranges"])
    assert bit_equal(O.domain_pool(g["signal"], p["tile"], rs, step), g["pool"])


@pytest.mark.parametrize("case", CASES)
def test_embedding_bitexact(case):
    """scipy's own DCT with numpy's BLAS norm orders (sdot: f32 products summed in f64)."""
    g = load(case)
    assert bit_equal(O.embed(g["pool"]), g["emb"])


@pytest.mark.parametrize("case", CASES)
def test_candidates_bitexact(case):
    """The reference's candidate rows exactly — order included: scores in its sgemv order, ties in numpy's order."""
    g = load(case)
    p = g["p"]
    pruned = O.range_energy_pruned(g["ranges"], p["thr"])
    for K in p["Ks"]:
        gold = g[f"cand_{K}"]
        assert np.array_equal(pruned, gold[:, 0] < 0)
        cand, _, _ = O.topk_candidates(g["emb"], len(gold), K, pruned, threads=8)
        assert np.array_equal(cand, gold)


@pytest.mark.parametrize("case", CASES)
def test_end_to_end_bitexact(case):
    """The oracle from the signal alone (voiced → ranges → pool → embeddings → search → affine) reproduces every
    match tuple of the reference."""
    g = load(case)
    p = g["p"]
    for K in p["Ks"]:
        r = O.compress(g["signal"], p["tile"], K, p["thr"])
        for nm in ("idx", "s", "o", "sym", "err"):
            assert bit_equal(r[nm], g[f"m_{nm}_{K}"]), nm


@pytest.mark.parametrize("case", CASES)
def test_affine_bitexact(case):
    g = load(case)
    for K in g["p"]["Ks"]:
        out = O.affine(g["ranges"], g[f"cand_{K}"], g["pool"])
        for nm, a in zip(("idx", "s", "o", "sym", "err"), out):
            assert bit_equal(a, g[f"m_{nm}_{K}"]), nm


@pytest.mark.parametrize("case", CASES)
def test_decode_bitexact(case):
    g = load(case)
    p = g["p"]
    for K in p["Ks"]:
        args = (g[f"m_idx_{K}"], g[f"m_s_{K}"], g[f"m_o_{K}"], g[f"m_sym_{K}"], g["pool"], len(g[f"m_idx_{K}"]),
                p["rs"])
        d, it, _ = O.decode(*args, original_len=p["original_len"])
        assert bit_equal(d, g[f"dec_{K}"]) and it == int(g[f"dec_iters_{K}"])
        d, _, _ = O.decode(*args, iterations=50, convergence_eps=0.0, original_len=p["original_len"])
        assert bit_equal(d, g[f"dec50_{K}"])
        d, it, dl = O.decode(*args, iterations=12, convergence_eps=0.0, s_damping=0.3, original_len=p["original_len"])
        assert bit_equal(d, g[f"decd_{K}"])
        np.testing.assert_allclose(dl, g[f"decd_deltas_{K}"], rtol=1e-5)
        # the reference's own Δ values (BLAS sdot norms) as its log prints them ({delta:.6e}, the goldens' source),
        # every one of them
        _, _, dr = O.decode(*args, iterations=12, convergence_eps=0.0, s_damping=0.3, deltas="reference")
        assert [float(f"{v:.6e}") for v in dr] == [float(v) for v in g[f"decd_deltas_{K}"]]
        _, _, dr = O.decode(*args, deltas="reference")
        assert [float(f"{v:.6e}") for v in dr] == [float(v) for v in g[f"dec_deltas_{K}"]]


@pytest.mark.parametrize("case", CASES)
def test_decode_early_exit_takes_reference_decision(case):
    """The stop decision is the reference's (Δ from numpy's BLAS sdot norms, fractal.py:1460-1465), not the float64
    measure's: with eps placed strictly between the two at an iteration where they differ, the oracle stops exactly
    where the reference's Δ says."""
    g = load(case)
    p = g["p"]
    K = max(p["Ks"])
    args = (g[f"m_idx_{K}"], g[f"m_s_{K}"], g[f"m_o_{K}"], g[f"m_sym_{K}"], g["pool"], len(g[f"m_idx_{K}"]), p["rs"])
    _, _, d64 = O.decode(*args, iterations=12, convergence_eps=0.0, s_damping=0.3)
    _, _, ref = O.decode(*args, iterations=12, convergence_eps=0.0, s_damping=0.3, deltas="reference")
    cand = [t for t in range(len(ref)) if ref[t] != d64[t] and all(ref[u] >= max(ref[t], d64[t]) for u in range(t))]
    if not cand:
        pytest.skip("no iteration where the two measures differ (and none before it is as small)")
    t = cand[0]
    lo, hi = sorted((ref[t], d64[t]))
    eps = (lo + hi) / 2
    _, it, _ = O.decode(*args, iterations=12, convergence_eps=eps, s_damping=0.3)
    assert it == (t + 1 if ref[t] < eps else min(12, next((u + 1 for u in range(t + 1, 12) if ref[u] < eps), 12)))


@pytest.mark.parametrize("case", [c for c in CASES if c in ("tone", "sweep", "ragged", "tiny")])
def test_fwav_bytes(case):
    g = load(case)
    p = g["p"]
    for K in p["Ks"]:
        b = O.fwav_bytes(g[f"m_idx_{K}"], g[f"m_s_{K}"], g[f"m_o_{K}"], g[f"m_sym_{K}"], g[f"m_err_{K}"], g["pool"],
                         p["rs"], p["framerate"], p["sampwidth"], p["tile"], p["step"], p["thr"], p["original_len"])
        assert b == g[f"fwav_{K}"].tobytes()


def test_pruned_ranges_emit_domain0_inf():
    """Quirk Q3: all-(-1) candidates → domain 0 (clamped) with s/o fitted to domain 0 and err=+inf."""
    g = load("speech4096")
    K = 64
    pr = g[f"cand_{K}"][:, 0] < 0
    assert pr.any()
    assert np.all(g[f"m_idx_{K}"][pr] == 0) and np.all(np.isinf(g[f"m_err_{K}"][pr]))


@pytest.mark.parametrize("case", CASES)
def test_embedding_heads_at_most_unit_norm(case):
    """The fp16 pre-filter's error bound δ (fwav_topk.hip kF16Delta) assumes every embedding head — tonal dims 0-7,
    transient dims 8-15 — has norm ≤ 1 (fractal.py:205-207, 161-163 normalise; zero rows stay zero)."""
    g = load(case)
    e = g["emb"].astype(np.float64)
    for head in (e[:, :8], e[:, 8:]):
        assert np.sqrt((head ** 2).sum(1)).max() <= 1 + 1e-6


def test_smooth_matches_numpy_convolve():
    """The voiced detection's moving average is np.convolve(e, ones(5)/5, 'same') (fractal.py:893-895); the oracle's
    restatement (and the device kernel that mirrors it) must equal numpy bit-for-bit on energies spanning many decades,
    where the order and precision of each window's sum matter — including fewer frames than taps, where numpy swaps
    the operands."""
    rng = np.random.default_rng(11)
    for w in (5, 3, 7):
        for _ in range(600):
            n = int(rng.integers(1, 40))
            e = (rng.random(n) * rng.choice([1e-5, 1e-2, 1.0, 1e3], n)).astype(np.float32)
            ref = np.convolve(e, np.full(w, np.float32(1) / np.float32(w), np.float32), mode="same")
            assert np.array_equal(O.smooth5(e, w).view(np.uint32), ref.view(np.uint32)), (w, n)


def _unit_head_rows(rng, nd):
    """Rows shaped like the reference's embeddings: tonal dims 0-7 and transient dims 8-15 each of unit norm."""
    e = rng.standard_normal((nd, 16)).astype(np.float32)
    for h in (slice(0, 8), slice(8, 16)):
        e[:, h] /= np.sqrt((e[:, h].astype(np.float64) ** 2).sum(1)).astype(np.float32)[:, None]
    return e


@pytest.mark.parametrize("nd", [28_801, 1_321_977])
def test_sgemv_thread_split_pinned_against_numpy(nd):
    """The reference's scores ``domain_embs @ q`` (fractal.py:537) above OpenBLAS's threading threshold
    (16·nd ≥ 460,800, i.e. nd ≥ 28,800: every config from cfg2 up): OpenBLAS splits the columns over its T threads and
    each thread scores its chunk's last columns with the 4x2 / 4x1 tail kernels.  The oracle's split
    (sgemv_col_kind) and per-kind order (sgemv_scores) must equal numpy's own ``E @ q`` bit-for-bit on every column
    for T ∈ {1, 2, 3, 5, 8, 16}, under threadpoolctl's limit — and fwav.ties.blas_threads() must read back that T
    from numpy's OpenBLAS.  A wrong T must be caught: the T = 1 split disagrees with numpy at T = 8."""
    threadpoolctl = pytest.importorskip("threadpoolctl")
    from fwav import ties

    rng = np.random.default_rng(nd)
    e = _unit_head_rows(rng, nd)
    qi = rng.integers(0, nd, 4)
    cols = np.arange(nd)
    refs = {}
    for T in (1, 2, 3, 5, 8, 16):
        with threadpoolctl.threadpool_limits(T, user_api="blas"):
            assert ties.blas_threads() == T
            assert O.blas_threads() == T
            refs[T] = np.stack([e @ e[i] for i in qi])
        got = O.sgemv_scores(e, e[qi], O.sgemv_col_kind(cols, nd, T))
        assert np.array_equal(got.view(np.uint32), refs[T].view(np.uint32)), (nd, T)
    if nd == 1_321_977:
        # the thread split is observable: scoring with T = 1's kernels misses numpy's T = 8 bits somewhere
        k1, k8 = O.sgemv_col_kind(cols, nd, 1), O.sgemv_col_kind(cols, nd, 8)
        assert (k1 != k8).sum() == 20
        wrong = O.sgemv_scores(e, e[qi], k1)
        assert not np.array_equal(wrong.view(np.uint32), refs[8].view(np.uint32))


@pytest.mark.parametrize("case", ["sweep", "noise2048", "speech4096"])
def test_full_size_row_checker_accepts_reference_rows(case):
    """tests/oracle_rows.check_rows (the full-size GPU parity check) accepts the reference's own candidate rows and
    match tuples, row subsets and large-table thresholds included, and rejects a row with two candidates swapped."""
    from oracle_rows import check_rows
    g = load(case)
    p = g["p"]
    K = max(p["Ks"])
    gold = g[f"cand_{K}"]
    rows = np.nonzero(gold[:, 0] >= 0)[0][::7]
    outs = tuple(g[f"m_{nm}_{K}"] for nm in ("idx", "s", "o", "sym", "err"))
    got = check_rows(g["emb"], g["pool"], g["ranges"], gold, outs, rows, K, 8, chunk=16, label=case)
    assert got["rows"] == len(rows)
    bad = gold.copy()
    tied = O.topk_rows(g["emb"], rows, K, 8)[3]
    r = int(rows[np.nonzero(~tied)[0][len(rows) // 3]])  # a row whose top K + 1 scores are distinct
    bad[r, [3, 4]] = bad[r, [4, 3]]
    with pytest.raises(AssertionError):
        check_rows(g["emb"], g["pool"], g["ranges"], bad, outs, [r], K, 8, label=case)


@pytest.mark.parametrize("n", [0, 1, 31, 32, 33, 63, 64, 65, 95, 96, 97, 127, 128, 129, 1000, 4097, 65537, 200003])
def test_sdot_blas_pinned(n):
    """O.sdot_blas (the order of np.linalg.norm's BLAS sdot, fractal.py:1460-1461) equals numpy's own x.dot(y) bit for
    bit, at 1 and 8 OpenBLAS threads (the single-threaded result is numpy's at any thread count)."""
    from threadpoolctl import threadpool_limits
    rng = np.random.default_rng(n)
    for trial in range(2):
        x = (rng.standard_normal(n) * np.exp(rng.uniform(-4, 4, n))).astype(np.float32)
        y = rng.standard_normal(n).astype(np.float32)
        for T in (1, 8):
            with threadpool_limits(T, user_api="blas"):
                for a, b in ((x, x), (x, y)):
                    want = a.dot(b) if n else np.float32(0)
                    assert O.sdot_blas(a, b).view(np.uint32) == np.float32(want).view(np.uint32), (n, T)


def test_cfg2_tuple_fixture_pinned():
    """tests/golden/cfg2_tuples_t16.npz (every cfg2 match tuple with 16 BLAS threads, make_cfg2_tuples.py) against
    the oracle recomputed here on 256 sampled untied rows plus 8 of its numpy-ranked tie rows: same embedding table
    (digest), same tuples bit for bit."""
    import hashlib
    import json
    import os

    import threadpoolctl

    from fwav import synth
    fx = np.load(os.path.join(os.path.dirname(__file__), "golden", "cfg2_tuples_t16.npz"))
    par = json.loads(str(fx["params"]))
    sig, _, _ = synth.make_config_signal("cfg2")
    rs, step = O.geometry(par["tile"])
    vm = O.voiced_detection(sig, 2 * rs, par["energy_thresh"])
    ranges, _ = O.form_ranges(sig, vm, rs)
    pool = O.domain_pool(sig, par["tile"], rs, step)
    emb = O.embed(pool)
    assert hashlib.sha256(emb.tobytes()).hexdigest() == str(fx["emb_sha256"])
    rng = np.random.default_rng(11)
    tied = fx["tie_rows"]
    rows = np.union1d(rng.choice(np.setdiff1d(np.arange(len(ranges)), tied), 256, replace=False),
                      rng.choice(tied, 8, replace=False))

    def row_scores(q):
        with threadpoolctl.threadpool_limits(par["blas_threads"]):
            return O.reference_row_scores(emb, q, par["blas_threads"])

    cand, _, _, _ = O.topk_rows(emb, rows, par["K"], par["blas_threads"], row_scores=row_scores)
    got = O.affine(ranges[rows], cand, pool)
    for nm, v in zip(("idx", "s", "o", "sym", "err"), got):
        assert np.array_equal(np.asarray(v).view(np.uint8), fx[nm][rows].view(np.uint8)), nm
