"""The reference's score order on the machine the product runs on, and the bounded device memory of the tie ranking.

* ``fwav_score_rows`` with the thread count ``fwav.ties.blas_threads()`` reads from numpy's own OpenBLAS must equal
  numpy's ``emb @ q`` (fractal.py:537) computed on this host, bit for bit, on the real cfg2 table (1,321,977 domains:
  above OpenBLAS's threading threshold, so its thread split decides which columns its tail kernels score).
* ``fwav.ties.rank_rows_async`` queues at most its budget of exact score rows on the device per slice, whatever the
  number of tied rows, and still returns numpy's ranking of every row.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from fwav import engine, synth, ties  # noqa: E402
from fwav._lib import call  # noqa: E402
from oracle import fractal_oracle as O  # noqa: E402

K = 64


def dev():
    return torch.device("cuda", 0)


@pytest.fixture(scope="module")
def cfg2_table():
    sig, _, _ = synth.make_config_signal("cfg2")
    res = engine.compress_device(torch.from_numpy(sig).to(dev()), 2048, K, shard=(0, 64), keep_intermediates=True,
                                 tie_order="index")
    torch.cuda.synchronize()
    return res


def test_cfg2_score_rows_equal_numpy_on_this_host(cfg2_table):
    res = cfg2_table
    nd = res.n_domains
    assert nd == 1_321_977 and 16 * nd >= O.SGEMV_THREAD_MIN_MN
    T = ties.blas_threads()
    import threadpoolctl
    info = [i for i in threadpoolctl.threadpool_info() if i.get("internal_api") == "openblas"]
    print(f"numpy's OpenBLAS: {T} threads; threadpoolctl {[(i['num_threads'], i['architecture']) for i in info]}")
    assert T in [i["num_threads"] for i in info]
    rng = np.random.default_rng(7)
    rows = np.concatenate([[0, 1, nd - 1], rng.choice(res.n_ranges, 61, replace=False)]).astype(np.int32)
    S = torch.empty(len(rows) * nd, dtype=torch.float32, device=dev())
    r_d = torch.from_numpy(rows).to(dev())
    call("fwav_score_rows", res.emb.data_ptr(), nd, r_d.data_ptr(), len(rows), 0, T, S.data_ptr(),
         torch.cuda.current_stream().cuda_stream)
    got = S.view(len(rows), nd).cpu().numpy()
    emb = res.emb.view(-1, 16).cpu().numpy()
    kinds = O.sgemv_col_kind(np.arange(nd), nd, T)
    print(f"tail-kernel columns at T={T}: {int((kinds == 1).sum())} (4x2), {int((kinds == 2).sum())} (4x1)")
    for j, r in enumerate(rows):
        ref = emb @ emb[r]  # numpy's own sgemv on this host, at its own thread count
        assert np.array_equal(got[j].view(np.uint32), ref.view(np.uint32)), (int(r), int((got[j] != ref).sum()))


def test_rank_rows_async_device_memory_is_bounded(cfg2_table):
    """200 tied rows of the cfg2 table (1.06 GB of score rows) through a 4-row (21 MB) budget: the device never holds
    more than one budget of score rows, and every row is numpy's own ranking of its exact score row."""
    res = cfg2_table
    nd = res.n_domains
    T = ties.blas_threads()
    n = 200
    rows = torch.arange(0, 2 * n, 2, dtype=torch.int32, device=dev())
    budget = 4 * 4 * nd
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    fut = ties.rank_rows_async(rows, emb=res.emb, n_domains=nd, q_offset=0, k=K, threads=T,
                               stream=torch.cuda.current_stream().cuda_stream, budget=budget)
    got = np.stack([f.result() for f in fut.result()])
    torch.cuda.synchronize()
    peak = torch.cuda.max_memory_allocated() - base
    print(f"{n} rows x {nd} domains through a {budget / 1e6:.1f} MB budget: peak {peak / 1e6:.1f} MB")
    assert peak <= budget + (2 << 20)
    emb = res.emb.view(-1, 16).cpu().numpy()
    kinds = O.sgemv_col_kind(np.arange(nd), nd, T)
    for j in (0, 1, 57, n - 1):
        r = int(rows[j])
        ref = O.numpy_topk_row(O.sgemv_scores(emb, emb[r][None, :], kinds)[0], K)
        assert np.array_equal(got[j], ref), r


def test_rank_rows_async_many_slices_bounded(cfg2_table, monkeypatch):
    """Several slices' rankings in flight at once (the sliced search queues one per slice before any finishes): the
    eager launches stop at PIPE_EAGER_TOTAL (here 2 budgets), the rest go through the driver's side stream one budget
    at a time, so the device peak stays ≈ PIPE_EAGER_TOTAL + one budget — and every row is still numpy's ranking."""
    res = cfg2_table
    nd = res.n_domains
    T = ties.blas_threads()
    budget = 4 * 4 * nd
    monkeypatch.setattr(ties, "PIPE_EAGER_TOTAL", 2 * budget)
    slices = [torch.arange(s0, s0 + 40, dtype=torch.int32, device=dev()) for s0 in range(0, 240, 40)]
    torch.cuda.synchronize()
    base = torch.cuda.memory_allocated()
    torch.cuda.reset_peak_memory_stats()
    futs = [ties.rank_rows_async(r, emb=res.emb, n_domains=nd, q_offset=0, k=K, threads=T,
                                 stream=torch.cuda.current_stream().cuda_stream, budget=budget) for r in slices]
    got = [np.stack([f.result() for f in fu.result()]) for fu in futs]
    torch.cuda.synchronize()
    peak = torch.cuda.max_memory_allocated() - base
    print(f"6 slices x 40 rows through {budget / 1e6:.1f} MB budgets: peak {peak / 1e6:.1f} MB")
    assert peak <= 3 * budget + (4 << 20)
    assert ties._EAGER_BYTES == 0
    emb = res.emb.view(-1, 16).cpu().numpy()
    kinds = O.sgemv_col_kind(np.arange(nd), nd, T)
    for j, r in ((0, 0), (3, 17), (5, 39)):
        q = int(slices[j][r])
        assert np.array_equal(got[j][r], O.numpy_topk_row(O.sgemv_scores(emb, emb[q][None, :], kinds)[0], K)), q
