"""Full-size parity at BASELINE.json's large configs, through properties that do not need the oracle to run the whole
search (the oracle's scalar top-K would take hours at these sizes):

* cfg3 (10 min speech-like @ 44.1 kHz, tile 4096: 1,653,750 ranges × 6,613,977 domains), the whole compress:
  voiced mask + ranges bit-exact vs the oracle over the whole signal; pool/embedding rows at the start, middle and
  end; the energy prune vs host energies; sampled queries' candidates are a top-K set of the exact scores (torch
  fp32 rescoring, ties within 1e-5) and equal the all-f32 kernel's, as does every active query's candidate row; affine bit-exact (oracle) on the sampled
  ranges; decode bit-exact (oracle) over all ranges.
* cfg4 (60 min @ 48 kHz, tile 2048: 86,398,977 domains — a 2.76 GB fp16 table, so table offsets pass 2^31): pool and
  embeddings at the end of the table, and a 2,048-range shard searched against the whole table (top-K property,
  affine bit-exact).
* cfg2 rank shares (the strong-scaling bench's per-rank work at 2 / 4 / 8 ranks): every candidate row of the
  default work plan (all blocks in table pieces) equals the all-f32 kernel's.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from fwav import engine, synth, ties  # noqa: E402
from fwav._lib import call, debug_library, size_call  # noqa: E402
from oracle import fractal_oracle as O  # noqa: E402
from oracle_rows import check_rows  # noqa: E402

pytestmark = pytest.mark.gpu
K = 64
SAMPLE = 32


def dev():
    return torch.device("cuda", 0)


def exact_scores(emb_t, q, chunk=1 << 22):
    """f64 elementwise scores, chunked.  Not `emb_t @ q`: torch's fp32 gemv (rocBLAS) returns garbage for the
    86.4 M × 16 cfg4 table (|Δ| up to 3.7e19 vs exact, tools/diag_large_nd.py), which our kernels do not."""
    q = q.double()
    out = torch.empty(emb_t.shape[0], dtype=torch.float64, device=emb_t.device)
    for a in range(0, emb_t.shape[0], chunk):
        out[a:a + chunk] = (emb_t[a:a + chunk].double() * q).sum(-1)
    return out


def check_topk_property(emb_t, qrow, cand_row, k, tol=1e-5):
    """cand_row holds k distinct domains whose exact scores all reach the k-th best score (up to tol)."""
    s = exact_scores(emb_t, emb_t[qrow])
    kth = torch.topk(s, k).values[-1].item()
    c = torch.from_numpy(np.asarray(cand_row, np.int64)).to(s.device)
    assert (c >= 0).all() and len(torch.unique(c)) == k
    assert s[c].min().item() >= kth - tol, (qrow, s[c].min().item(), kth)


def f32_search(res, rows, k):
    """The all-f32 MFMA kernel on a subset of the shard's queries (local indices `rows`)."""
    m = res.shard[1] - res.shard[0]
    act = torch.from_numpy(np.asarray(rows, np.int32)).to(dev())
    n = torch.tensor([len(rows)], dtype=torch.int32, device=dev())
    cand = torch.full((m * k,), -7, dtype=torch.int32, device=dev())
    call("fwav_sim_topk", res.emb.data_ptr(), None, res.n_domains, act.data_ptr(), n.data_ptr(), len(rows),
         res.shard[0], k, ties.blas_threads(), cand.data_ptr(), None, None, 0, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    return cand.view(m, k)[act.long()].cpu().numpy()


@pytest.fixture(scope="module")
def cfg3_both():
    """cfg3 compressed twice: with the device's (score desc, index asc) order for exact ties — what the all-f32
    kernel returns — and with the product default, numpy's order on the rows where it changes a match."""
    sig, sr, _ = synth.make_config_signal("cfg3")
    x = torch.from_numpy(sig).to(dev())
    res = engine.compress_device(x, 4096, K, keep_intermediates=True, tie_order="index")
    prod = engine.compress_device(x, 4096, K, keep_intermediates=True)
    torch.cuda.synchronize()
    return sig, res, prod


@pytest.fixture(scope="module")
def cfg3(cfg3_both):
    return cfg3_both[:2]


def test_cfg3_geometry_ranges_pool(cfg3):
    sig, res = cfg3
    assert (res.n_ranges, res.n_domains, res.range_size) == (1653750, 6613977, 16)
    mask = O.voiced_detection(sig, 2 * 16)
    ranges, _ = O.form_ranges(sig, mask, 16)
    assert np.array_equal(res.ranges.cpu().numpy().view(np.uint32), ranges.reshape(-1).view(np.uint32))
    pool = res.pool.view(-1, 16)
    emb = res.emb.view(-1, 16)
    step, tile, nd = 4, 4096, res.n_domains
    for d0 in (0, nd // 2, nd - 2048):
        seg = sig[d0 * step:(d0 + 2047) * step + tile]
        p = O.domain_pool(seg, tile, 16, step)[:2048]
        assert np.array_equal(pool[d0:d0 + 2048].cpu().numpy().view(np.uint32), p.view(np.uint32))
        # bit-exact embeddings (scipy's pocketfft sequence), −60 dBFS pause tiles included
        assert np.array_equal(emb[d0:d0 + 2048].cpu().numpy().view(np.uint32), O.embed(p).view(np.uint32))
    # the fp16 pre-filter's δ assumes every head of every table row has norm ≤ 1 (fwav_topk.hip kF16Delta)
    heads = emb.double().view(-1, 2, 8).square().sum(-1).sqrt()
    assert float(heads.max()) <= 1 + 1e-6


def test_cfg3_prune_and_search(cfg3):
    sig, res = cfg3
    ranges = res.ranges.view(-1, 16).cpu().numpy()
    pruned = O.range_energy_pruned(ranges, 1e-4)
    cand = res.cand.view(-1, K)
    first = cand[:, 0].cpu().numpy()
    assert np.array_equal(first < 0, pruned)
    assert int(res.n_active.item()) == int((~pruned).sum())
    assert 0.2 < pruned.mean() < 0.9  # the speech-like generator prunes its pauses
    rng = np.random.default_rng(3)
    rows = np.sort(rng.choice(np.nonzero(~pruned)[0], SAMPLE, replace=False))
    emb_t = res.emb.view(-1, 16)
    got = cand[torch.from_numpy(rows).to(dev())].cpu().numpy()
    for r, c in zip(rows, got):
        check_topk_property(emb_t, int(r), c, K)
    assert np.array_equal(f32_search(res, rows, K), got)


def test_cfg3_f16_equals_f32_every_query(cfg3):
    """The whole cfg3 search (666,606 active queries; ≈ 35% overflow the fp16 band and take the exact-mode
    relaunch) returns exactly the all-f32 kernel's candidates for every query."""
    sig, res = cfg3
    cand = res.cand.view(-1, K)
    rows = np.nonzero(cand[:, 0].cpu().numpy() >= 0)[0]
    assert len(rows) == int(res.n_active.item())
    ref = f32_search(res, rows, K)
    got = cand[torch.from_numpy(rows).to(dev())].cpu().numpy()
    assert np.array_equal(ref, got), int((ref != got).any(axis=1).sum())


def test_cfg3_numpy_tie_order(cfg3_both):
    """The product's tie handling at full size: rows outside the resolved list equal the index-order run; every
    resolved row is numpy's own ranking of the reference-order score row (oracle.sgemv_scores over the whole 6.6 M
    domain table, numpy_topk_row) and its tuple the oracle's affine of that row."""
    sig, res, prod = cfg3_both
    print(f"cfg3: {prod.n_ties} queries with exact ties in their top K + 1, {prod.n_resolved} re-ranked by numpy")
    a = res.cand.view(-1, K).cpu().numpy()
    b = prod.cand.view(-1, K).cpu().numpy()
    diff = np.nonzero((a != b).any(axis=1))[0]
    assert len(diff) <= prod.n_resolved
    emb = prod.emb.view(-1, 16).cpu().numpy()
    nd = prod.n_domains
    kinds = O.sgemv_col_kind(np.arange(nd), nd, ties.blas_threads())
    pool = prod.pool.view(-1, 16).cpu().numpy()
    ranges = prod.ranges.view(-1, 16).cpu().numpy()
    for r in diff[:6]:
        ref = O.numpy_topk_row(O.sgemv_scores(emb, emb[r][None, :], kinds)[0], K)
        assert np.array_equal(b[r], ref), r
        out = O.affine(ranges[r:r + 1], ref[None, :], pool)
        for t, v in zip((prod.idx, prod.s, prod.o, prod.sym, prod.err), out):
            assert np.array_equal(t[r:r + 1].cpu().numpy().view(np.uint8), np.asarray(v).view(np.uint8))
    # K-th place ties the tie check left in index order (every member of the tied group fits worse than the best
    # candidate outside it): numpy's own ranking gives the same match tuple
    rec = prod.ties[1:1 + 9 * prod.n_ties].view(-1, 9).cpu().numpy()
    kept = [int(e >> 1) for e in rec[:, 0] if (e & 1) and int(e >> 1) not in set(diff.tolist())]
    print(f"cfg3: {int((rec[:, 0] & 1).sum())} K-th place ties, {len(kept)} left in index order")
    assert len(kept) > 0
    for r in kept[:8]:
        ref = O.numpy_topk_row(O.sgemv_scores(emb, emb[r][None, :], kinds)[0], K)
        out = O.affine(ranges[r:r + 1], ref[None, :], pool)
        for t, v in zip((prod.idx, prod.s, prod.o, prod.sym, prod.err), out):
            assert np.array_equal(t[r:r + 1].cpu().numpy().view(np.uint8), np.asarray(v).view(np.uint8)), r


def test_cfg3_candidate_rows_equal_oracle(cfg3_both):
    """≥ 256 sampled active rows of the product-default cfg3 search (plus 32 of the rows it lists with exact ties)
    against the oracle's rows in the reference's sgemv order for this process's BLAS threads (fractal.py:535-541):
    order included wherever numpy's order decides it, and every match tuple = O.affine of the oracle's row
    (tests/oracle_rows.py)."""
    sig, _, prod = cfg3_both
    T = ties.blas_threads()
    emb = prod.emb.view(-1, 16).cpu().numpy()
    pool = prod.pool.view(-1, 16).cpu().numpy()
    ranges = prod.ranges.view(-1, 16).cpu().numpy()
    cand = prod.cand.view(-1, K).cpu().numpy()
    outs = tuple(t.cpu().numpy() for t in (prod.idx, prod.s, prod.o, prod.sym, prod.err))
    active = np.nonzero(cand[:, 0] >= 0)[0]
    rec = prod.ties[1:1 + engine.TIE_REC * prod.n_ties].view(-1, engine.TIE_REC).cpu().numpy()
    listed = np.unique(rec[:, 0] >> 1)
    rng = np.random.default_rng(33)
    rows = np.union1d(rng.choice(active, 256, replace=False), rng.choice(listed, min(32, len(listed)), replace=False))
    got = check_rows(emb, pool, ranges, cand, outs, rows, K, T, exact=prod.resolved.cpu().numpy(), chunk=32,
                     label="cfg3 defaults")
    assert got["rows"] >= 256 and got["tied"] > 0


def test_cfg3_affine_sampled(cfg3):
    sig, res = cfg3
    ranges = res.ranges.view(-1, 16).cpu().numpy()
    cand = res.cand.view(-1, K).cpu().numpy()
    rng = np.random.default_rng(4)
    rows = np.sort(rng.choice(res.n_ranges, 4096, replace=False))
    pool = res.pool.view(-1, 16).cpu().numpy()
    a = O.affine(ranges[rows], cand[rows], pool)
    for t, b in zip((res.idx, res.s, res.o, res.sym, res.err), a):
        got = t.cpu().numpy()[rows]
        assert np.array_equal(got.view(np.uint8), np.asarray(b).view(np.uint8))


def test_cfg3_decode_bitexact(cfg3):
    sig, res = cfg3
    rec, ran, _ = engine.decompress_device(res.idx, res.s, res.o, res.sym, res.pool, res.n_ranges, 16)
    d, it, _ = O.decode(res.idx.cpu().numpy(), res.s.cpu().numpy(), res.o.cpu().numpy(), res.sym.cpu().numpy(),
                        res.pool.view(-1, 16).cpu().numpy(), res.n_ranges, 16)
    assert ran == it
    assert np.array_equal(rec.cpu().numpy().view(np.uint32), d.reshape(-1).view(np.uint32))


def test_cfg4_table_end_and_shard_search():
    sig, sr, _ = synth.make_config_signal("cfg4")
    n = sig.size
    rs, step, tile = 8, 2, 2048
    nr = -(-n // rs)
    lo = nr // 2
    res = engine.compress_device(torch.from_numpy(sig).to(dev()), tile, K, shard=(lo, lo + 2048),
                                 keep_intermediates=True, tie_order="index")
    torch.cuda.synchronize()
    nd = res.n_domains
    assert nd == 86398977 and res.n_ranges == nr
    assert (nd * 16 * 2) > 2 ** 31  # the fp16 table's byte offsets exceed 32 bits
    pool = res.pool.view(-1, rs)
    emb_t = res.emb.view(-1, 16)
    d0 = nd - 4096
    seg = sig[d0 * step:(d0 + 4095) * step + tile]
    p = O.domain_pool(seg, tile, rs, step)[:4096]
    assert np.array_equal(pool[d0:].cpu().numpy().view(np.uint32), p.view(np.uint32))
    assert np.array_equal(emb_t[d0:].cpu().numpy().view(np.uint32), O.embed(p).view(np.uint32))
    cand = res.cand.view(-1, K).cpu().numpy()
    assert (cand[:, 0] >= 0).all()  # noise: nothing pruned
    for j in range(0, 2048, 128):
        check_topk_property(emb_t, lo + j, cand[j], K)
    ranges = res.ranges.view(-1, rs)[lo:lo + 2048].cpu().numpy()
    a = O.affine(ranges, cand, pool.cpu().numpy())
    for t, b in zip((res.idx, res.s, res.o, res.sym, res.err), a):
        assert np.array_equal(t.cpu().numpy().view(np.uint8), np.asarray(b).view(np.uint8))


@pytest.mark.parametrize("world", [2, 4, 8])
def test_cfg2_rank_share_equals_f32(world):
    """One rank's share of the full cfg2 search (the strong-scaling bench's per-rank work): its default work plan
    splits every query block into table pieces merged by k_merge_pieces (pieces share their band limits), so this
    is the product path at its real piece counts — every candidate row must equal the all-f32 kernel's."""
    sig, _, _ = synth.make_config_signal("cfg2")
    nr = -(-sig.size // 8)
    lo, hi = (world - 1) * nr // world, nr  # the last rank's block (a shard not starting at 0)
    res = engine.compress_device(torch.from_numpy(sig).to(dev()), 2048, K, shard=(lo, hi), keep_intermediates=True,
                                 tie_order="index")
    torch.cuda.synchronize()
    cand = res.cand.view(-1, K).cpu().numpy()
    assert cand.shape[0] == hi - lo and (cand >= 0).all() and (cand < res.n_domains).all()
    ref = f32_search(res, np.arange(hi - lo), K)
    assert np.array_equal(cand, ref)


def test_cfg2_whole_search_equals_f32():
    """The whole cfg2 search (1,292 query blocks on 512 workgroup slots, the tail in table pieces) equals the all-f32
    kernel on every row."""
    sig, _, _ = synth.make_config_signal("cfg2")
    res = engine.compress_device(torch.from_numpy(sig).to(dev()), 2048, K, keep_intermediates=True, tie_order="index")
    torch.cuda.synchronize()
    cand = res.cand.view(-1, K).cpu().numpy()
    assert (cand >= 0).all() and (cand < res.n_domains).all()
    assert np.array_equal(cand, f32_search(res, np.arange(res.n_ranges), K))


def test_cfg4_shard_wide_geometry_default():
    """A cfg4 shard of 337,500 consecutive queries (one rank's share of 64) against the whole 86.4 M-domain table —
    where the centroid filter in the wide geometry (16 waves × 2 sets of 32 queries, one workgroup per CU) is the
    default first pass.  The plan is asserted to be that one with whole-table blocks; every row equals the
    base-geometry search (8 waves, no centroids, a different plan and processing order), 1,024 rows equal the all-f32
    kernel, and sampled rows hold the exact top K (fractal.py:535-541)."""
    sig, _, _ = synth.make_config_signal("cfg4", seed=0)
    q = 337_500
    x = torch.from_numpy(sig).to(dev())
    res = engine.compress_device(x, 2048, K, shard=(0, q), keep_intermediates=True, tie_order="index")
    torch.cuda.synchronize()
    nd = res.n_domains
    info = np.zeros(3, np.int32)
    blocks = np.zeros(3, np.int64)
    with debug_library():
        call("fwav_debug_topk_plan_info", q, nd, info.ctypes.data, blocks.ctypes.data)
    print(f"cfg4 shard plan: wide {info[0]} mode {info[1]} pieces {info[2]} whole blocks {blocks[0]} split "
          f"{blocks[1]} grid {blocks[2]}")
    # the centroid filter in the wide geometry: 330 blocks of 1,024 queries on 256 slots, every block in table pieces
    assert info[0] == 3 and blocks[0] + blocks[1] == -(-q // 1024) and blocks[2] >= blocks[0] + blocks[1]
    wide = res.cand.view(-1, K).cpu().numpy()
    assert (wide >= 0).all() and (wide < nd).all()
    with debug_library():
        call("fwav_debug_topk_geometry", 0)
        base = engine.compress_device(x, 2048, K, shard=(0, q), keep_intermediates=True, tie_order="index")
        torch.cuda.synchronize()
    assert np.array_equal(wide, base.cand.view(-1, K).cpu().numpy())
    rows = np.arange(0, q, q // 1024)[:1024]
    assert np.array_equal(wide[rows], f32_search(res, rows, K))
    emb_t = res.emb.view(-1, 16)
    for j in rows[::128]:
        check_topk_property(emb_t, int(j), wide[j], K)
