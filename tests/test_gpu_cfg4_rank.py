"""cfg4 (BASELINE configs[3]: 60 min @ 48 kHz noise, tile 2048, K 64, ranges sharded over 8 GPUs) at its per-rank size:
one rank's eighth — 2,700,000 queries against the whole 86,398,977-domain table — through the product path exactly
as a rank of the 8-GPU compress runs it (fwav.engine.compress_device with shard=, the product defaults: the sliced
search over ≥ 4 Mi-domain tables, numpy's tie order with each slice's tied rows ranked while the next slice searches).
Reference: the range split fractal.py:1180-1182, cpu_worker :556-632, range_candidates_from_embedding_emb :535-541,
_process_gpu_batch :757-850.

Checked against properties that do not need the oracle's whole search (which would take days on the host):
  * candidate rows equal the all-f32 kernel's on 16,384 sampled rows (rows re-ranked by numpy excepted: the f32
    kernel returns the device's (score desc, index asc) order among exactly equal scores);
  * sampled rows hold the exact top K (f64 rescoring on the device, ties within 1e-5);
  * the first 6 numpy-ranked rows equal the oracle's ranking of the oracle's reference-order score row
    (O.numpy_topk_row(O.sgemv_scores(...)), computed in column chunks);
  * every match tuple of 4,096 sampled ranges (the ranked rows among them) is the oracle's affine solve of its
    candidate row, bit for bit.
"""
import time

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from fwav import engine, synth, ties  # noqa: E402
from fwav._lib import call  # noqa: E402
from oracle import fractal_oracle as O  # noqa: E402
from oracle_rows import check_rows  # noqa: E402

pytestmark = pytest.mark.gpu
K = 64
EIGHTH = 2_700_000


def dev():
    return torch.device("cuda", 0)


def oracle_row(emb: np.ndarray, q: np.ndarray, threads: int, chunk: int = 1 << 23) -> np.ndarray:
    """The reference's score row emb @ q in its sgemv order (O.sgemv_scores), in column chunks (bounded memory)."""
    nd = len(emb)
    out = np.empty(nd, np.float32)
    for a in range(0, nd, chunk):
        cols = np.arange(a, min(nd, a + chunk))
        out[a:a + len(cols)] = O.sgemv_scores(emb[a:a + len(cols)], q[None, :], O.sgemv_col_kind(cols, nd, threads))[0]
    return out


def test_cfg4_one_rank_eighth_product_path():
    sig, _, _ = synth.make_config_signal("cfg4")
    n = sig.size
    rs, step, tile = 8, 2, 2048
    nr = -(-n // rs)
    assert nr == 21_600_000
    lo, hi = nr - EIGHTH, nr  # the last rank's block (a shard far from offset 0)
    x = torch.from_numpy(sig).to(dev())
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = engine.compress_device(x, tile, K, shard=(lo, hi), keep_intermediates=True)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    nd = res.n_domains
    assert nd == 86_398_977
    nsub = engine._tie_sub_blocks(EIGHTH, nd)
    print(f"cfg4 rank eighth: {EIGHTH} queries x {nd} domains in {wall:.2f} s ({nsub} search slices); "
          f"{res.n_ties} queries with exact ties in their top K + 1, {res.n_resolved} ranked by numpy")
    assert nsub > 1  # the sliced path
    cand = res.cand.view(-1, K)
    T = ties.blas_threads()
    # the rows numpy re-ranked: the tie list's rows whose product row differs from the device order are a subset
    rng = np.random.default_rng(44)
    rows = np.sort(rng.choice(EIGHTH, 16_384, replace=False)).astype(np.int32)
    act = torch.from_numpy(rows).to(dev())
    n_act = torch.tensor([len(rows)], dtype=torch.int32, device=dev())
    ref = torch.full((EIGHTH * K,), -7, dtype=torch.int32, device=dev())
    call("fwav_sim_topk", res.emb.data_ptr(), None, nd, act.data_ptr(), n_act.data_ptr(), len(rows), lo, K, T,
         ref.data_ptr(), None, None, 0, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = cand[act.long()].cpu().numpy()
    ref = ref.view(-1, K)[act.long()].cpu().numpy()
    assert (got >= 0).all() and (got < nd).all()
    diff = np.nonzero((got != ref).any(axis=1))[0]
    rec = res.ties[1:1 + 9 * res.n_ties].view(-1, 9).cpu().numpy()
    tied = set((rec[:, 0] >> 1).tolist())
    assert all(int(rows[i]) in tied for i in diff), "a row without exact ties differs from the all-f32 kernel"
    # same candidate set wherever only the order of equal scores moved
    assert len(diff) <= res.n_resolved
    emb_t = res.emb.view(-1, 16)
    for i in range(0, len(rows), 2048):
        r = int(rows[i])
        q = emb_t[lo + r].double()
        sc = torch.empty(nd, dtype=torch.float64, device=dev())
        for a in range(0, nd, 1 << 24):
            sc[a:a + (1 << 24)] = (emb_t[a:a + (1 << 24)].double() * q).sum(-1)
        kth = torch.topk(sc, K).values[-1].item()
        c = torch.from_numpy(got[i].astype(np.int64)).to(dev())
        assert len(torch.unique(c)) == K and sc[c].min().item() >= kth - 1e-5, r
    # numpy's own ranking of the reference-order score row, on the first numpy-ranked rows
    emb = res.emb.view(-1, 16).cpu().numpy()
    pool = res.pool.view(-1, rs).cpu().numpy()
    ranges = res.ranges.view(-1, rs)[lo:hi].cpu().numpy()
    cand_h = cand.cpu().numpy()
    ranked = res.resolved.cpu().numpy()
    assert len(ranked) == res.n_resolved > 0
    for r in ranked[:6]:
        want = O.numpy_topk_row(oracle_row(emb, emb[lo + r], T), K)
        assert np.array_equal(want, cand_h[r]), int(r)
        out = O.affine(ranges[r:r + 1], want[None, :], pool)
        for t, v in zip((res.idx, res.s, res.o, res.sym, res.err), out):
            assert np.array_equal(t[r:r + 1].cpu().numpy().view(np.uint8), np.asarray(v).view(np.uint8)), int(r)
    checked = min(6, len(ranked))
    # the affine solve of sampled ranges (and of every row above) bit-exact
    samp = np.sort(rng.choice(EIGHTH, 4096, replace=False))
    out = O.affine(ranges[samp], cand_h[samp], pool)
    for t, v in zip((res.idx, res.s, res.o, res.sym, res.err), out):
        assert np.array_equal(t.cpu().numpy()[samp].view(np.uint8), np.asarray(v).view(np.uint8))
    # ≥ 64 sampled rows (and 8 of the listed tie rows) against the oracle's rows, order included where numpy's order
    # decides it, and their match tuples = O.affine of the oracle's rows (tests/oracle_rows.py)
    rec_rows = np.unique(rec[:, 0] >> 1)
    orows = np.union1d(rng.choice(EIGHTH, 64, replace=False), rng.choice(rec_rows, min(8, len(rec_rows)), replace=False))
    outs_h = tuple(t.cpu().numpy() for t in (res.idx, res.s, res.o, res.sym, res.err))
    got_o = check_rows(emb, pool, ranges, cand_h, outs_h, orows, K, T, q_offset=lo, exact=ranked, chunk=8,
                       label="cfg4 rank eighth")
    assert got_o["rows"] >= 64
    print(f"cfg4 rank eighth: 16,384 rows = f32 kernel (numpy-ranked rows aside: {len(diff)}), top-K property on "
          f"8 rows, {checked} tie rows = numpy's ranking of the reference row, 4,096 tuples = oracle; "
          f"product call {wall:.2f} s")
