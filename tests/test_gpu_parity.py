"""GPU parity: the HIP path (through the C-ABI) against the reference goldens and the oracle.

Bars: the whole compress bit-exact with the reference on every golden case — ranges, voiced mask, pool, embeddings
(scipy's own pocketfft sequence), candidate sets (the reference's BLAS score order, numpy's order among exactly tied
scores wherever it can change a match), every (domain_index, s, o, symmetry_flag, err) tuple, the .fwav bytes — and
the decode bit-exact.
"""
import numpy as np
import pytest

from golden_util import CASES, bit_equal, load

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from fwav import engine  # noqa: E402
from fwav._lib import call, debug_library  # noqa: E402


def dev():
    return torch.device("cuda", 0)


def td(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev())


def run_case(g, K, tie_order="numpy"):
    p = g["p"]
    res = engine.compress_device(td(g["signal"]), p["tile"], K, energy_thresh=p["thr"], keep_intermediates=True,
                                 tie_order=tie_order)
    torch.cuda.synchronize()
    return res


@pytest.mark.parametrize("case", CASES)
def test_ranges_pool_embed(case):
    g = load(case)
    K = g["p"]["Ks"][0] if g["p"]["Ks"][0] <= 64 else 32
    r = run_case(g, K)
    rs = g["p"]["rs"]
    assert bit_equal(r.ranges.cpu().numpy().reshape(-1, rs), g["ranges"])
    assert bit_equal(r.pool.cpu().numpy().reshape(-1, rs), g["pool"])
    emb = r.emb.cpu().numpy().reshape(-1, 16)
    assert bit_equal(emb, g["emb"])


@pytest.mark.parametrize("case", CASES)
def test_candidates_and_matches(case):
    """With tie_order="numpy_sets": the reference's candidate set for every range and its order wherever the top-K
    scores are distinct (among exactly equal scores the device keeps index order unless numpy's order can change the
    match — fwav.ties), and every match tuple bit-exact (SURVEY Appendix A rules 3-4 at their strictest: no
    exceptions).  The product default (tie_order="numpy", K-th place ties re-ranked only where they can decide the
    match) gives the same tuples."""
    from oracle import fractal_oracle as O
    g = load(case)
    p = g["p"]
    for K in p["Ks"]:  # includes ragged K=2000 >= n_domains (full sort, −1 padded)
        d = run_case(g, K)
        for nm, t in (("idx", d.idx), ("s", d.s), ("o", d.o), ("sym", d.sym), ("err", d.err)):
            assert bit_equal(t.cpu().numpy(), g[f"m_{nm}_{K}"]), f"{case} K={K} {nm} (default tie order)"
        r = run_case(g, K, "numpy_sets")
        cand = r.cand.cpu().numpy().reshape(-1, K)
        gold = g[f"cand_{K}"]
        assert all(set(a.tolist()) == set(b.tolist()) for a, b in zip(cand, gold)), f"{case} K={K}: candidate sets"
        # order: equal wherever the golden row's scores are all distinct
        emb = g["emb"]
        for i in range(len(gold)):
            c = gold[i][gold[i] >= 0]
            if len(c) == 0:
                continue
            sc = O.sgemv_scores(emb[c], emb[i][None, :], O.sgemv_col_kind(c, len(emb), 8))[0]
            if len(np.unique(sc)) == len(sc):
                assert np.array_equal(cand[i], gold[i]), f"{case} K={K} row {i}"
        for nm, t in (("idx", r.idx), ("s", r.s), ("o", r.o), ("sym", r.sym), ("err", r.err)):
            assert bit_equal(t.cpu().numpy(), g[f"m_{nm}_{K}"]), f"{case} K={K} {nm}"
        print(f"{case} K={K}: {r.n_ties} rows with exact ties, {r.n_resolved} re-ranked by numpy for the sets, "
              f"{d.n_resolved} for the matches; all tuples exact")


@pytest.mark.parametrize("case", CASES)
def test_affine_bitexact_on_golden_candidates(case):
    g = load(case)
    p = g["p"]
    rs = p["rs"]
    for K in p["Ks"]:
        cand = g[f"cand_{K}"]
        nr = len(cand)
        out = [torch.empty(nr, dtype=dt, device=dev()) for dt in
               (torch.int32, torch.float32, torch.float32, torch.uint8, torch.float32)]
        ranges, c, pool = td(g["ranges"].reshape(-1)), td(cand.reshape(-1)), td(g["pool"].reshape(-1))
        call("fwav_affine", ranges.data_ptr(), nr, rs, c.data_ptr(), K, pool.data_ptr(), len(g["pool"]), 16.0,
             *[t.data_ptr() for t in out], torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        for nm, t in zip(("idx", "s", "o", "sym", "err"), out):
            assert bit_equal(t.cpu().numpy(), g[f"m_{nm}_{K}"]), f"{case} K={K} {nm}"


@pytest.mark.parametrize("case", CASES)
def test_decode_bitexact(case):
    from fwav.api import decompress_audio
    from fwav.matches import MatchList
    g = load(case)
    p = g["p"]
    for K in p["Ks"]:
        m = MatchList(g[f"m_idx_{K}"], g[f"m_s_{K}"], g[f"m_o_{K}"], g[f"m_sym_{K}"], g[f"m_err_{K}"])
        nr = len(m)
        d, info = decompress_audio(m, g["pool"], nr, p["rs"], original_len=p["original_len"], return_info=True)
        assert bit_equal(d, g[f"dec_{K}"])
        assert info["iterations"] == int(g[f"dec_iters_{K}"])
        d = decompress_audio(m, g["pool"], nr, p["rs"], iterations=50, convergence_eps=0.0,
                             original_len=p["original_len"])
        assert bit_equal(d, g[f"dec50_{K}"])
        d, info = decompress_audio(m, g["pool"], nr, p["rs"], iterations=12, convergence_eps=0.0, s_damping=0.3,
                                   original_len=p["original_len"], return_info=True)
        assert bit_equal(d, g[f"decd_{K}"])
        np.testing.assert_allclose(info["deltas"], g[f"decd_deltas_{K}"], rtol=1e-5)


def test_reference_e2e_tone(tmp_path):
    """The reference's own test (test_e2e.py:13-38), unmodified in substance (batch_size= alias accepted)."""
    import fractal
    from fwav import synth
    sig, sr, sw = synth.tone(), 8000, 2
    matches, domains, n_ranges, range_size, tile_size, domain_step, energy_thresh, orig_len = fractal.compress_audio(
        sig, sr, sw, tile_size=128, energy_thresh=1e-4, use_gpu=False, domains_tmpdir=str(tmp_path), batch_size=32,
        fast_mode=True)
    assert len(matches) == n_ranges
    assert domains.shape[1] == range_size
    fw = tmp_path / "test_e2e.fwav"
    fractal.save_compressed(str(fw), matches, domains, range_size, sr, sw, tile_size, domain_step, energy_thresh,
                            len(sig))
    m2, d2, nr2, rs2, fr2, sw2, t2, ds2, et2, ol2 = fractal.load_compressed(str(fw))
    recon = fractal.decompress_audio(m2, d2, nr2, rs2, iterations=8, convergence_eps=1e-3, use_gpu=False,
                                     original_len=ol2)
    snr = fractal.compute_snr(sig, np.asarray(recon))
    assert snr > 4.0
    g = load("tone")
    assert len(matches) == len(g["m_idx_32"])
    # the .fwav written here is the reference's file byte for byte (fractal.py:1278-1322: header, SHA-256 of the
    # body, pool, 17-byte match records) — the tone's byte-identical tiles included, whose matches follow numpy's
    # order among exactly tied scores
    assert np.array_equal(np.frombuffer(fw.read_bytes(), np.uint8), g["fwav_32"])


def _cands(sig, tile, K, search, thr=1e-4, tie_order="numpy_sets"):
    r = engine.compress_device(td(sig), tile, K, energy_thresh=thr, keep_intermediates=True, search=search,
                               tie_order=tie_order)
    torch.cuda.synchronize()
    return r.cand.cpu().numpy().reshape(-1, K), r


@pytest.fixture(params=[(-1, -1), (0, 0), (1, 0), (0, 1), (1, 1), (0, 2), (1, 2), (0, 3), (1, 3)],
                ids=["auto", "s16-base", "hl-base", "s16-wide", "hl-wide", "s16-cent", "hl-cent", "s16-centw",
                     "hl-centw"])
def first_mode(request):
    """Run a test under each first-pass mode (fwav_debug_topk_mode) and workgroup geometry (fwav_debug_topk_geometry)
    of the fp16 search, then restore the defaults."""
    mode, wide = request.param
    with debug_library():  # the knobs exist in libfwav_debug.so only; the whole test runs through it
        call("fwav_debug_topk_mode", mode)
        call("fwav_debug_topk_geometry", wide)
        yield mode


@pytest.mark.parametrize("case", CASES)
def test_f16_prefilter_equals_f32_search(case, first_mode):
    """The fp16 pre-filter kernel must select exactly the f32 kernel's candidates (same order)."""
    g = load(case)
    for K in g["p"]["Ks"]:
        if K > 64:
            continue
        a, ra = _cands(g["signal"], g["p"]["tile"], K, "f16")
        b, rb = _cands(g["signal"], g["p"]["tile"], K, "f32")
        assert np.array_equal(a, b)
        for x, y in ((ra.idx, rb.idx), (ra.s, rb.s), (ra.o, rb.o), (ra.sym, rb.sym), (ra.err, rb.err)):
            assert bit_equal(x.cpu().numpy(), y.cpu().numpy())


@pytest.mark.parametrize("gen,tile,K", [("noise", 2048, 64), ("speech", 4096, 64), ("noise", 1024, 32),
                                        ("speech", 2048, 17)])
def test_f16_prefilter_equals_f32_larger(gen, tile, K, first_mode):
    from fwav import synth
    sig = synth.noise(6.0, 44100, seed=11) if gen == "noise" else synth.speech_like(6.0, 44100, seed=5)
    a, _ = _cands(sig, tile, K, "f16")
    b, _ = _cands(sig, tile, K, "f32")
    assert np.array_equal(a, b)


def _periodic(n=24000, period=96):
    """Period 96 (not a divisor of the 256-sample pool blocks at tile 1024, so block means — and embeddings — are not
    constant; a period of 32 would make every embedding zero, quirk Q11): every domain has ≈ nd/96 exact duplicates."""
    t = np.arange(n)
    return np.round(8000 * np.sin(2 * np.pi * t / period) + 3000 * np.sin(2 * np.pi * 3 * t / period)
                    ).astype(np.float32)


def test_f16_band_overflow_falls_back_to_exact(first_mode):
    """Massive exact ties (≈ 240 equal scores per query) overflow the fp16 band of the key buffer; those queries are
    searched again in exact mode (seeded with the first pass's band limit) — results must stay identical to the
    all-f32 kernel."""
    sig = _periodic()
    a, r = _cands(sig, 1024, 32, "f16")
    b, _ = _cands(sig, 1024, 32, "f32")
    emb = r.emb.cpu().numpy().reshape(-1, 16)
    assert not np.all(emb == 0, axis=1).any()
    assert (emb @ emb[0] == (emb @ emb[0]).max()).sum() > 192  # more ties than the band's 192 slots
    assert np.array_equal(a, b)


@pytest.mark.parametrize("gen,tile", [("noise", 2048), ("speech", 4096), ("periodic", 1024)])
def test_large_k_prefix_equals_k64(gen, tile):
    """K > 64 runs the batched score-row + select kernels; its first 64 columns must be exactly the K=64
    result (same score chain, same (score desc, index asc) order).  The periodic signal has ~nd/96 exactly
    tied scores per query, which defeats the sampled threshold and exercises the radix-select fallback.  Compared in
    the device's own order (tie_order="index"): numpy's order among exactly equal scores depends on K."""
    from fwav import synth
    sig = {"noise": lambda: synth.noise(3.0, 44100, seed=3), "speech": lambda: synth.speech_like(3.0, 44100, seed=4),
           "periodic": _periodic}[gen]()
    a, r = _cands(sig, tile, 64, "f32", tie_order="index")
    zeroq = np.all(r.emb.cpu().numpy().reshape(-1, 16)[:len(a)] == 0, axis=1)
    for K in (65, 200, 1000):
        b, _ = _cands(sig, tile, K, "f16", tie_order="index")
        # zero queries take the reference's introselect order for THIS K (quirk Q11), not a prefix of K = 64's
        assert np.array_equal(b[:, :64][~zeroq], a[~zeroq]), f"{gen} K={K}"
        assert (b[zeroq] == engine.zero_query_candidates(r.n_domains, K)).all()
        act = (b[:, 0] >= 0) & ~zeroq
        assert act.sum() > 1000
        assert (b[act] >= 0).all()
        assert all(len(set(row.tolist())) == K for row in b[act][:200])


@pytest.mark.parametrize("K", [65, 300, 1000])
def test_large_k_vs_oracle(K):
    """K > 64 (batched score rows + select): candidate sets equal the oracle's (the reference's numpy calls on the
    reference-order scores) for every range, and every match tuple equals the oracle's."""
    from oracle import fractal_oracle as orc

    g = load("noise2048")
    p = g["p"]
    r = run_case(g, K)
    cand = r.cand.cpu().numpy().reshape(-1, K)
    pruned = cand[:, 0] < 0
    ocand, _, _ = orc.topk_candidates(g["emb"], p["n_ranges"], K, pruned, threads=8)
    assert all(set(a.tolist()) == set(b.tolist()) for a, b in zip(cand, ocand))
    out = orc.affine(g["ranges"], ocand, g["pool"])
    for t, b in zip((r.idx, r.s, r.o, r.sym, r.err), out):
        assert bit_equal(t.cpu().numpy(), np.asarray(b))


@pytest.mark.parametrize("wide", [0, 1, 2, 3], ids=["base", "wide", "cent", "centw"])
@pytest.mark.parametrize("plan", [(0, 1), (1 << 20, 2), (1 << 20, 5), (1 << 20, 8), (10, 3), (1 << 20, -1), (7, -1)])
def test_f16_split_plans_equal_f32(plan, wide):
    """Work plans that split query blocks into table pieces (merged by k_merge_pieces) or into query halves return
    exactly the unsplit search's candidates: whole, all blocks in 2/5/8 pieces, only the last 10 blocks in 3, and all /
    the last 7 blocks as two half-blocks (4 waves each; the other waves exit at once)."""
    from fwav import synth
    sig = synth.noise(6.0, 44100, seed=11)
    b, _ = _cands(sig, 2048, 64, "f32")
    with debug_library():
        call("fwav_debug_topk_plan", *plan)
        call("fwav_debug_topk_geometry", wide)
        a, _ = _cands(sig, 2048, 64, "f16")
        p, _ = _cands(_periodic(), 1024, 32, "f16")  # band overflow inside pieces → exact-mode relaunch after the merge
    assert np.array_equal(a, b)
    q, _ = _cands(_periodic(), 1024, 32, "f32")
    assert np.array_equal(p, q)


def test_overflow_with_sparse_active_list(first_mode):
    """max_q bounds the number of listed queries, not their indices: a short active list of large local indices on a
    signal whose fp16 bands overflow must keep the overflow bookkeeping inside the workspace (guard bytes after it
    stay untouched) and return the all-f32 kernel's candidates."""
    from fwav import engine as E
    from fwav._lib import sim_topk_layout, size_call
    sig = td(_periodic(192_000))  # ≈ 2,000 exact copies per query: > 192 even in each of 8 table pieces
    tile, K = 1024, 32
    rs, step = E.geometry(tile)
    nd = (sig.numel() - tile) // step + 1
    st = torch.cuda.current_stream().cuda_stream
    tab = E.embed_tables(rs, sig.device)
    pool = torch.empty(nd * rs, device=sig.device)
    emb = torch.empty(nd * 16, device=sig.device)
    emb16 = torch.empty(2 * ((nd + 255) // 256) * 256 * 16, dtype=torch.float16, device=sig.device)
    ws = torch.empty(max(size_call("fwav_pool_workspace_size", sig.numel(), tile, rs, step), 16), dtype=torch.uint8,
                     device=sig.device)
    call("fwav_pool_embed", sig.data_ptr(), sig.numel(), tile, rs, step, tab.data_ptr(), pool.data_ptr(),
         emb.data_ptr(), emb16.data_ptr(), ws.data_ptr(), ws.numel(), st)
    n = nd // 2                                     # local queries 0 .. n−1 have cand rows
    rows = torch.arange(n - 300, n, dtype=torch.int32, device=sig.device)  # indices far above max_q
    max_q = len(rows)
    n_act = torch.tensor([max_q], dtype=torch.int32, device=sig.device)
    out = []
    for e16 in (emb16.data_ptr(), None):
        wsn = size_call("fwav_sim_topk_workspace_size", max_q, nd, K)
        guard = 1 << 20
        wsk = torch.zeros(wsn + guard, dtype=torch.uint8, device=sig.device)
        cand = torch.full((n * K,), -7, dtype=torch.int32, device=sig.device)
        call("fwav_sim_topk", emb.data_ptr(), e16, nd, rows.data_ptr(), n_act.data_ptr(), max_q, 0, K, 1,
             cand.data_ptr(), None, wsk.data_ptr(), wsn, st)
        torch.cuda.synchronize()
        assert int(wsk[wsn:].count_nonzero().item()) == 0, "write past the workspace"
        out.append(cand.view(n, K)[rows.long()].cpu().numpy())
        if e16 is not None:  # the first pass's overflow count (the library's own layout): the exact path ran
            o = sim_topk_layout(max_q, nd)["n_ovf1"]
            assert int(wsk[o:o + 4].view(torch.int32).item()) > 0
    assert np.array_equal(out[0], out[1])


def test_active_list_order_does_not_change_candidates():
    """The centroid geometry searches its own ascending copy of the active list (order_active): the same
    41,344 queries listed ascending, in fwav_prune's kind of order (runs of 64 in random run order), descending, and
    with every id listed twice (duplicates collapse) give the same candidate rows — and those of the all-f32 kernel —
    with the workspace untouched past its end; a list holding an id past max_q is searched as given."""
    from fwav import engine as E
    from fwav import synth
    from fwav._lib import size_call
    sig = td(synth.noise(60.0, 44100, seed=3))
    tile, K = 2048, 64
    rs, step = E.geometry(tile)
    nd = (sig.numel() - tile) // step + 1
    st = torch.cuda.current_stream().cuda_stream
    tab = E.embed_tables(rs, sig.device)
    pool = torch.empty(nd * rs, device=sig.device)
    emb = torch.empty(nd * 16, device=sig.device)
    emb16 = torch.empty(2 * ((nd + 255) // 256) * 256 * 16, dtype=torch.float16, device=sig.device)
    ws = torch.empty(max(size_call("fwav_pool_workspace_size", sig.numel(), tile, rs, step), 16), dtype=torch.uint8,
                     device=sig.device)
    call("fwav_pool_embed", sig.data_ptr(), sig.numel(), tile, rs, step, tab.data_ptr(), pool.data_ptr(),
         emb.data_ptr(), emb16.data_ptr(), ws.data_ptr(), ws.numel(), st)
    nq = 41_344
    lo = 100_000
    g = torch.Generator().manual_seed(1)
    runs = torch.randperm((nq + 63) // 64, generator=g).tolist()
    asc = torch.arange(nq, dtype=torch.int32)
    lists = {"ascending": asc,
             "runs": torch.cat([asc[r * 64:(r + 1) * 64] for r in runs]),
             "descending": asc.flip(0),
             "duplicates": torch.cat([asc, asc])}
    out = {}
    for name, lst in lists.items():
        for e16 in ((emb16.data_ptr(),) if name != "ascending" else (emb16.data_ptr(), None)):
            act = lst.to(sig.device)
            max_q = act.numel()
            n_act = torch.tensor([max_q], dtype=torch.int32, device=sig.device)
            wsn = size_call("fwav_sim_topk_workspace_size", max_q, nd, K)
            guard = 1 << 20
            wsk = torch.zeros(wsn + guard, dtype=torch.uint8, device=sig.device)
            cand = torch.full((max_q * K,), -7, dtype=torch.int32, device=sig.device)
            call("fwav_sim_topk", emb.data_ptr(), e16, nd, act.data_ptr(), n_act.data_ptr(), max_q, lo, K, 16,
                 cand.data_ptr(), None, wsk.data_ptr(), wsn, st)
            torch.cuda.synchronize()
            assert int(wsk[wsn:].count_nonzero().item()) == 0, f"{name}: write past the workspace"
            out[(name, e16 is None)] = cand.view(max_q, K)[:nq].cpu().numpy()
    ref = out[("ascending", True)]  # the all-f32 kernel
    for key, c in out.items():
        assert np.array_equal(c, ref), key
    # ids past max_q (33,344 ≥ 32,768 listed: the centroid geometry): the list is searched as given
    act = torch.arange(8_000, nq, dtype=torch.int32, device=sig.device).flip(0)
    max_q = act.numel()
    n_act = torch.tensor([max_q], dtype=torch.int32, device=sig.device)
    wsn = size_call("fwav_sim_topk_workspace_size", max_q, nd, K)
    wsk = torch.zeros(wsn, dtype=torch.uint8, device=sig.device)
    cand = torch.full((nq * K,), -7, dtype=torch.int32, device=sig.device)
    call("fwav_sim_topk", emb.data_ptr(), emb16.data_ptr(), nd, act.data_ptr(), n_act.data_ptr(), max_q, lo, K, 16,
         cand.data_ptr(), None, wsk.data_ptr(), wsn, st)
    torch.cuda.synchronize()
    assert np.array_equal(cand.view(nq, K)[8_000:].cpu().numpy(), ref[8_000:])


@pytest.mark.parametrize("n", [1, 7, 8, 127, 128, 129, 8191, 8192, 8193, 100_003, 2_646_000])
def test_weighted_energy_is_numpy_f32_sum(n):
    """The silent-input test's Σ x² (fractal.py:1083) equals np.sum(x ** 2) on float32 bit-for-bit."""
    rng = np.random.default_rng(n)
    x = (rng.normal(0, 1e-3, n) * rng.random(n)).astype(np.float32)
    t = td(x)
    from fwav._lib import size_call
    out = torch.empty(1, dtype=torch.float32, device=dev())
    wn = size_call("fwav_weighted_energy_workspace_size", n)
    ws = torch.empty(wn, dtype=torch.uint8, device=dev())
    call("fwav_weighted_energy", t.data_ptr(), n, out.data_ptr(), ws.data_ptr(), wn,
         torch.cuda.current_stream().cuda_stream)
    assert bit_equal(out.cpu().numpy(), np.array([np.sum(x ** 2)], np.float32))


def test_gather_rows_diagnostic_runs():
    """fwav_debug_gather_rows (the bench's random-row ceiling for the affine solve) runs on every supported row width
    and rejects unsupported ones."""
    from fwav._lib import FwavError
    st = torch.cuda.current_stream().cuda_stream
    sink = torch.zeros(1, dtype=torch.float32, device=dev())
    for rs in (4, 8, 16):
        tab = torch.rand(100_003 * rs, dtype=torch.float32, device=dev())
        call("fwav_debug_gather_rows", tab.data_ptr(), 100_003, rs, 1 << 18, sink.data_ptr(), st)
    torch.cuda.synchronize()
    with pytest.raises(FwavError):
        call("fwav_debug_gather_rows", tab.data_ptr(), 100_003, 5, 16, sink.data_ptr(), st)


@pytest.mark.parametrize("w", [5, 3, 7])
def test_smoothing_equals_numpy_convolve(w):
    """fwav_voiced_ranges' moving average (fwav_debug_smooth exposes it) equals np.convolve(e, ones(w)/w, 'same')[:nf]
    bit-for-bit on energies spanning many decades — full windows in f32, edge windows as numpy's f64-accumulated dot,
    and fewer frames than taps (numpy swaps the operands)."""
    rng = np.random.default_rng(w)
    st = torch.cuda.current_stream().cuda_stream
    for _ in range(200):
        nf = int(rng.integers(1, 40))
        e = (rng.random(nf) * rng.choice([1e-5, 1e-2, 1.0, 1e3], nf)).astype(np.float32)
        ref = np.convolve(e, np.full(w, np.float32(1) / np.float32(w), np.float32), mode="same")[:nf]
        et = td(e)
        out = torch.empty(nf, dtype=torch.float32, device=dev())
        call("fwav_debug_smooth", et.data_ptr(), nf, w, out.data_ptr(), st)
        assert bit_equal(out.cpu().numpy(), ref), (w, nf)


def test_half_of_41344_queries_pieces_plan_stays_in_workspace():
    """Regression for round 2's memory fault (tools/phase_ab.py): 20,672 queries against the full cfg2 table run the
    table-pieces plan (every block split, shared limits, k_merge_pieces).  With the workspace sized exactly for that
    query count, nothing is written past it (1 MiB guard), every emitted index is a domain, and the rows equal the
    all-f32 kernel's."""
    from fwav import synth
    from fwav import engine as E
    from fwav._lib import size_call
    sig = td(synth.noise(60.0, 44100, seed=0))
    tile, K = 2048, 64
    rs, step = E.geometry(tile)
    nd = (sig.numel() - tile) // step + 1
    st = torch.cuda.current_stream().cuda_stream
    tab = E.embed_tables(rs, sig.device)
    pool = torch.empty(nd * rs, device=sig.device)
    emb = torch.empty(nd * 16, device=sig.device)
    emb16 = torch.empty(2 * ((nd + 255) // 256) * 256 * 16, dtype=torch.float16, device=sig.device)
    ws = torch.empty(max(size_call("fwav_pool_workspace_size", sig.numel(), tile, rs, step), 16), dtype=torch.uint8,
                     device=sig.device)
    call("fwav_pool_embed", sig.data_ptr(), sig.numel(), tile, rs, step, tab.data_ptr(), pool.data_ptr(),
         emb.data_ptr(), emb16.data_ptr(), ws.data_ptr(), ws.numel(), st)
    rows = torch.arange(0, 41344, 2, dtype=torch.int32, device=sig.device)  # the even half, as phase_ab's A
    max_q = rows.numel()
    n_act = torch.tensor([max_q], dtype=torch.int32, device=sig.device)
    out = []
    for e16 in (emb16.data_ptr(), None):
        wsn = size_call("fwav_sim_topk_workspace_size", max_q, nd, K)
        guard = 1 << 20
        wsk = torch.zeros(wsn + guard, dtype=torch.uint8, device=sig.device)
        cand = torch.full((41344 * K,), -7, dtype=torch.int32, device=sig.device)
        call("fwav_sim_topk", emb.data_ptr(), e16, nd, rows.data_ptr(), n_act.data_ptr(), max_q, 0, K, 1,
             cand.data_ptr(), None, wsk.data_ptr(), wsn, st)
        torch.cuda.synchronize()
        assert int(wsk[wsn:].count_nonzero().item()) == 0, "write past the workspace"
        c = cand.view(-1, K)[rows.long()].cpu().numpy()
        assert ((c >= 0) & (c < nd)).all()
        out.append(c)
    assert np.array_equal(out[0], out[1])


def _adversarial_emb(nd, seed):
    """Unit-head embedding rows built to stress the fp16 hi/lo split (DESIGN §3.1 δ′ bound): components exactly
    halfway between fp16 neighbours (x_hi rounds to even, x_lo is a whole half-ulp), components below 2^-14 (fp16
    subnormal x_hi) and below 2^-3 (fp16-subnormal x_lo); heads brought to norm ≤ 1 by exact halvings; every third
    row a near-duplicate of another (one component moved by one fp16 ulp), which packs scores near the K-th."""
    rng = np.random.default_rng(seed)
    E = np.empty((nd, 16), np.float32)
    j = np.arange(8)
    for h in (0, 1):
        kind = rng.integers(0, 3, nd)[:, None]
        mant = rng.integers(0, 1024, (nd, 8))
        mid = np.ldexp(1024.0 + mant + 0.5, rng.integers(-6, 0, (nd, 8)) - 10)
        tiny = np.where(j % 2 == 1, np.ldexp(1.0 + rng.random((nd, 8)), -15 - (j % 9)), np.ldexp(1024.0 + mant + 0.5, -11))
        small = np.ldexp(rng.random((nd, 8)), -4 - (j % 3))
        x = np.where(kind == 0, mid, np.where(kind == 1, tiny, small)) * np.where(rng.random((nd, 8)) < 0.5, -1.0, 1.0)
        k = np.maximum(0, np.ceil(np.log2(np.maximum((x * x).sum(1), 1e-300)) / 2)).astype(np.int64)
        E[:, 8 * h:8 * h + 8] = np.ldexp(x, -k[:, None]).astype(np.float32)
    dup = np.arange(0, nd, 3)
    E[dup] = E[rng.integers(0, nd, len(dup))]
    E[dup, rng.integers(0, 16, len(dup))] *= np.float32(0.99951171875)
    assert (np.sqrt((E[:, :8].astype(np.float64) ** 2).sum(1)) <= 1).all()
    assert (np.sqrt((E[:, 8:].astype(np.float64) ** 2).sum(1)) <= 1).all()
    return E


@pytest.mark.parametrize("K", [64, 17])
def test_hilo_band_adversarial_embeddings(K, first_mode):
    """The fp16 search in every first-pass mode (the hi/lo band above all) returns the all-f32 kernel's candidates on
    embeddings built to break the hi/lo error bound (fp16 midpoints, fp16-subnormal hi and lo parts, near-duplicate
    rows): the band margins δ = 2e-3 / δ′ = 1e-5 hold there too."""
    from fwav._lib import size_call
    nd, nq = 60_000, 4096
    E = _adversarial_emb(nd, 7)
    emb = td(E.reshape(-1))
    st = torch.cuda.current_stream().cuda_stream
    emb16 = torch.empty(size_call("fwav_emb16_elems", nd), dtype=torch.float16, device=dev())
    call("fwav_emb16_from_emb", emb.data_ptr(), nd, emb16.data_ptr(), st)
    act = torch.arange(nq, dtype=torch.int32, device=dev())
    n_act = torch.tensor([nq], dtype=torch.int32, device=dev())
    out = []
    for e16 in (emb16.data_ptr(), None):
        wsn = size_call("fwav_sim_topk_workspace_size", nq, nd, K)
        wsk = torch.empty(max(wsn, 16), dtype=torch.uint8, device=dev())
        cand = torch.full((nq * K,), -7, dtype=torch.int32, device=dev())
        call("fwav_sim_topk", emb.data_ptr(), e16, nd, act.data_ptr(), n_act.data_ptr(), nq, 0, K, 1,
             cand.data_ptr(), None, wsk.data_ptr(), wsn, st)
        torch.cuda.synchronize()
        out.append(cand.view(nq, K).cpu().numpy())
    assert ((out[1] >= 0) & (out[1] < nd)).all()
    assert np.array_equal(out[0], out[1])


def test_deferred_tie_resolution_equals_synchronous():
    """defer_ties=True (the bench's pipelined mode): the host half of the tie resolution runs on the driver thread
    while later calls are queued; after wait() every output equals the synchronous call's, for several calls in
    flight at once (tone, K = 32: its byte-identical tiles give rows that numpy re-ranks)."""
    g = load("tone")
    p = g["p"]
    sig = td(g["signal"])
    ref = engine.compress_device(sig, p["tile"], 32, energy_thresh=p["thr"], keep_intermediates=True)
    torch.cuda.synchronize()
    assert ref.n_resolved > 0
    outs = [engine.compress_device(sig, p["tile"], 32, energy_thresh=p["thr"], keep_intermediates=True,
                                   defer_ties=True) for _ in range(3)]
    for r in outs:
        r.wait()
    torch.cuda.synchronize()
    for r in outs:
        assert (r.n_ties, r.n_resolved) == (ref.n_ties, ref.n_resolved)
        for nm in ("cand", "idx", "s", "o", "sym", "err"):
            assert bit_equal(getattr(r, nm).cpu().numpy(), getattr(ref, nm).cpu().numpy()), nm


@pytest.mark.parametrize("nsub", [2, 5])
def test_sub_block_search_equals_single_launch(nsub):
    """sub_blocks=n (the search as n launches over slices of the active list, each slice's tied rows ranked on the
    host while the next slice searches — the default for large searches over ≥ 4 Mi-domain tables): every output,
    the tie counts and the candidate rows equal the single launch's (tone, K = 32: rows that numpy re-ranks; speech:
    pruned ranges, so slices hold uneven parts of the active list)."""
    for name, k in (("tone", 32), ("speech4096", 64), ("speech4096", 100)):  # K = 100: the large-K kernels
        g = load(name)
        p = g["p"]
        sig = td(g["signal"])
        ref = engine.compress_device(sig, p["tile"], k, energy_thresh=p["thr"], keep_intermediates=True,
                                     sub_blocks=1)
        got = engine.compress_device(sig, p["tile"], k, energy_thresh=p["thr"], keep_intermediates=True,
                                     sub_blocks=nsub)
        # deferred: the slices' rankings applied by wait()
        dfr = engine.compress_device(sig, p["tile"], k, energy_thresh=p["thr"], sub_blocks=nsub, defer_ties=True)
        dfr.wait()
        torch.cuda.synchronize()
        assert (dfr.n_ties, dfr.n_resolved) == (ref.n_ties, ref.n_resolved), name
        for nm in ("idx", "s", "o", "sym", "err"):
            assert bit_equal(getattr(dfr, nm).cpu().numpy(), getattr(ref, nm).cpu().numpy()), (name, "deferred", nm)
        if name == "tone":
            assert ref.n_resolved > 0
        assert (got.n_ties, got.n_resolved) == (ref.n_ties, ref.n_resolved), name
        for nm in ("cand", "idx", "s", "o", "sym", "err"):
            assert bit_equal(getattr(got, nm).cpu().numpy(), getattr(ref, nm).cpu().numpy()), (name, nm)
        # the slices' tie lists, merged, name the single launch's queries and boundary flags (records land in
        # completion order: compare sorted)
        def recs(r):
            t = r.ties.cpu().numpy()
            return np.sort(t[1:1 + 9 * int(t[0])].reshape(-1, 9)[:, 0])
        assert np.array_equal(recs(got), recs(ref)), name
        # a shard that starts mid-signal (a rank's block: query rows offset by lo)
        lo, hi = ref.n_ranges // 5, ref.n_ranges - ref.n_ranges // 7
        a = engine.compress_device(sig, p["tile"], k, energy_thresh=p["thr"], shard=(lo, hi), sub_blocks=1)
        b = engine.compress_device(sig, p["tile"], k, energy_thresh=p["thr"], shard=(lo, hi), sub_blocks=nsub)
        torch.cuda.synchronize()
        assert (a.n_ties, a.n_resolved) == (b.n_ties, b.n_resolved), name
        for nm in ("idx", "s", "o", "sym", "err"):
            assert bit_equal(getattr(b, nm).cpu().numpy(), getattr(a, nm).cpu().numpy()), (name, "shard", nm)
            assert bit_equal(getattr(b, nm).cpu().numpy(), getattr(ref, nm).cpu().numpy()[lo:hi]), (name, "rows", nm)


def test_pieces_plan_with_fewer_active_queries_than_launched():
    """The search's grid and workspace cover the plan of max_q, while every workgroup re-derives the plan from the
    device-side active count.  In the piece-major plan (every block split) the items past the smaller plan must do
    nothing: the same active list searched with max_q = 11,025 and with max_q = its own count gives identical rows
    (44 vs 20 blocks in 8 table pieces)."""
    from fwav import synth
    from fwav._lib import size_call
    sig = td(synth.noise(2.0, 44100, seed=3))
    from fwav import ties
    r = engine.compress_device(sig, 2048, 64, keep_intermediates=True, tie_order="index")
    torch.cuda.synchronize()
    nd, nr = r.n_domains, r.n_ranges
    st = torch.cuda.current_stream().cuda_stream
    emb16 = torch.empty(size_call("fwav_emb16_elems", nd), dtype=torch.float16, device=dev())
    call("fwav_emb16_from_emb", r.emb.data_ptr(), nd, emb16.data_ptr(), st)
    nq = 5000
    active = torch.arange(nq, dtype=torch.int32, device=dev())
    n_active = torch.tensor([nq], dtype=torch.int32, device=dev())
    out = {}
    for max_q in (nr, nq):
        wk = size_call("fwav_sim_topk_workspace_size", max_q, nd, 64)
        ws = torch.empty(wk, dtype=torch.uint8, device=dev())
        cand = torch.full((max_q * 64,), -7, dtype=torch.int32, device=dev())
        call("fwav_sim_topk", r.emb.data_ptr(), emb16.data_ptr(), nd, active.data_ptr(), n_active.data_ptr(), max_q,
             0, 64, ties.blas_threads(), cand.data_ptr(), None, ws.data_ptr(), wk, st)
        torch.cuda.synchronize()
        out[max_q] = cand[:nq * 64].cpu().numpy()
    assert np.array_equal(out[nr], out[nq])
    assert (out[nq] >= 0).all() and (out[nq] < nd).all()
    assert np.array_equal(out[nq].reshape(nq, 64), r.cand.view(-1, 64)[:nq].cpu().numpy())
