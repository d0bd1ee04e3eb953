"""GPU decode (fwav_decode.hip) against the oracle's decompress_audio restatement (fractal.py:1378-1473).

The iteration-resident kernel runs up to 64 iterations per launch with each range's reconstruction in registers and
recomputes the stopping chunk, so these cases cover: a stop inside the second chunk, forced runs across
chunk boundaries (64, 65, 130 iterations), every range_size bucket (exact 4/8/16/32, guarded 5/12/20/31) and the
streaming path (range_size > 32), sentinel −1 indices and constant tiles (‖T − mean T‖² = 0).  Bar: recon bit-exact,
the same iteration count, Δ within 1e-12 relative of the oracle's f64 measure (different order from numpy's) —
except at an iteration the exact early-exit check decided, which reports the reference's own float32 Δ.  The stop
decision itself is always the reference's (Δ from numpy's BLAS sdot norms, fractal.py:1460-1465): the last tests
place eps inside the certified band on both sides of the reference's Δ, single device and sharded.
"""
import numpy as np
import pytest

from golden_util import bit_equal, load

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from fwav import engine  # noqa: E402
from oracle import fractal_oracle as O  # noqa: E402


def td(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(torch.device("cuda", 0))


def synth_matches(nr, nd, rs, seed):
    rng = np.random.default_rng(seed)
    pool = rng.normal(0, 0.3, (nd, rs)).astype(np.float32)
    pool[::97] = 0.25  # constant tiles: den = 0 → not valid, s_stored kept
    idx = rng.integers(0, nd, nr).astype(np.int32)
    idx[::53] = -1  # sentinels (legacy path, fractal.py:1399-1426)
    s = rng.uniform(-1.2, 1.2, nr).astype(np.float32)
    o = rng.normal(0, 0.1, nr).astype(np.float32)
    sym = (rng.random(nr) < 0.5).astype(np.uint8)
    return idx, s, o, sym, pool


def check(idx, s, o, sym, pool, rs, **kw):
    nr = len(idx)
    rec, ran, deltas = engine.decompress_device(td(idx), td(s), td(o), td(sym), td(pool.reshape(-1)), nr, rs, **kw)
    ref, it, rdel = O.decode(idx, s, o, sym, pool, nr, rs, **kw)
    _, _, dref = O.decode(idx, s, o, sym, pool, nr, rs, deltas="reference", **kw)
    assert ran == it, (ran, it)
    assert bit_equal(rec.cpu().numpy(), ref)
    for a, b, c in zip(deltas, rdel, dref):  # f64 measure, or the reference's own Δ where the check decided
        assert a == c or abs(a - b) <= 1e-12 * abs(b), (a, b, c)
    return ran


@pytest.mark.parametrize("case", ["noise2048", "speech4096", "sweep"])
def test_stop_inside_second_chunk(case):
    g = load(case)
    K = g["p"]["Ks"][0]
    args = (g[f"m_idx_{K}"], g[f"m_s_{K}"], g[f"m_o_{K}"], g[f"m_sym_{K}"], g["pool"], g["p"]["rs"])
    ran = check(*args, iterations=300, convergence_eps=1e-6, s_damping=0.9)
    assert 64 < ran < 128


@pytest.mark.parametrize("iters", [1, 63, 64, 65, 130])
def test_forced_iterations_across_chunks(iters):
    idx, s, o, sym, pool = synth_matches(10_000, 3_000, 8, seed=iters)
    assert check(idx, s, o, sym, pool, 8, iterations=iters, convergence_eps=0.0, s_damping=0.5) == iters
    assert check(idx, s, o, sym, pool, 8, iterations=iters, convergence_eps=0.0) == iters


@pytest.mark.parametrize("rs", [4, 5, 8, 12, 16, 20, 31, 32, 40])
def test_every_range_size(rs):
    idx, s, o, sym, pool = synth_matches(9_000 + rs, 2_000, rs, seed=rs)
    check(idx, s, o, sym, pool, rs)                                              # defaults: stops at 2
    check(idx, s, o, sym, pool, rs, iterations=70, convergence_eps=1e-5, s_damping=0.7)
    check(idx, s, o, sym, pool, rs, iterations=5, convergence_eps=0.0, s_clip=0.5, s_damping=0.2)


def test_zero_iterations_and_empty():
    idx, s, o, sym, pool = synth_matches(100, 50, 8, seed=1)
    rec, ran, _ = engine.decompress_device(td(idx), td(s), td(o), td(sym), td(pool.reshape(-1)), 100, 8, iterations=0)
    assert ran == 0 and np.all(rec.cpu().numpy() == 0) and rec.numel() == 800


def _shard_decode(idx, s, o, sym, pool, rs, bounds, iterations, eps, s_damping=0.0):
    """Run the sharded C-ABI sequence for every shard on one device, adding the shards' partials the way the
    all-reduce of fwav.dist.decompress_sharded does, with its exact early-exit check (fwav.dist.decode_shard):
    → per shard (local reconstruction, iterations run, deltas)."""
    import torch as _t
    from fwav import dist
    nr = len(idx)
    decs = [dist.ShardDecoder(td(idx[a:b]), td(s[a:b]), td(o[a:b]), td(sym[a:b]), td(pool.reshape(-1)), a, nr, rs,
                              iterations, eps, 16.0, s_damping) for a, b in bounds]
    done, deltas = 0, []
    while True:
        for c in range(decs[0].n_chunks):
            for d in decs:
                d.run(c)
            tot = sum(d.partials_prefix() for d in decs)
            for d in decs:
                d.partials_prefix().copy_(tot)
                d.reduce(c)
        outs = [d.finish() for d in decs]
        ran = outs[0][1]
        assert all(o_[1] == ran and o_[2] == outs[0][2] for o_ in outs)
        done += ran
        deltas += outs[0][2]
        if outs[0][3] is None:
            break
        d_ref, stop = decs[0].exact_delta(_t.cat([o_[3] for o_ in outs]), _t.cat([o_[0] for o_ in outs]))
        deltas[-1] = d_ref
        if stop or done >= iterations:
            break
        decs = [d.resumed(o_[0], iterations - done) for d, o_ in zip(decs, outs)]
    return [(o_[0], done, deltas) for o_ in outs]


@pytest.mark.parametrize("world", [2, 3, 5])
def test_sharded_decode_bit_identical_to_single(world):
    """Shard bounds on multiples of fwav_decode_span(): the concatenated reconstruction, the iteration count and
    every Δ equal the single-device decode bit-for-bit (the Δ sums have one canonical order)."""
    from fwav import dist
    idx, s, o, sym, pool = synth_matches(50_000, 8_000, 8, seed=world)
    nr = len(idx)
    bounds = dist.decode_bounds(nr, world)
    assert bounds[0][0] == 0 and bounds[-1][1] == nr
    for iters, eps, damp in ((8, 1e-3, 0.0), (150, 1e-6, 0.9), (70, 0.0, 0.3)):
        rec1, ran1, del1 = engine.decompress_device(td(idx), td(s), td(o), td(sym), td(pool.reshape(-1)), nr, 8,
                                                    iterations=iters, convergence_eps=eps, s_damping=damp)
        outs = _shard_decode(idx, s, o, sym, pool, 8, bounds, iters, eps, damp)
        rec = np.concatenate([r.cpu().numpy() for r, _, _ in outs])
        assert bit_equal(rec, rec1.cpu().numpy())
        for _, ran, dl in outs:
            assert ran == ran1 and np.array_equal(np.asarray(dl), np.asarray(del1))


@pytest.mark.parametrize("n", [0, 1, 31, 32, 33, 64, 96, 97, 4_097, 262_144 + 33, 3_000_000 + 7])
def test_exact_delta_kernel_equals_reference(n):
    """fwav_decode_exact (one workgroup, the sdot's 64 accumulators as sequential fma chains) returns the reference's
    Δ = ‖next − prev‖ / (‖prev‖ or 1) with numpy's own norms (fractal.py:1460-1461) bit for bit."""
    rng = np.random.default_rng(n)
    prev = (rng.standard_normal(n) * np.exp(rng.uniform(-3, 3, n))).astype(np.float32)
    nxt = (prev + rng.standard_normal(n).astype(np.float32) * np.float32(0.01)).astype(np.float32)
    if n == 1:
        prev[:] = 0  # ‖prev‖ = 0: the reference divides by 1.0
    for p_, q_ in ((prev, nxt), (prev, prev)):
        st = td(np.array([2, 0, 0, 0], np.int32))
        d = td(np.zeros(1))
        from fwav._lib import call
        dp, dq = td(p_), td(q_)  # held: a temporary's memory would be handed to the next allocation
        call("fwav_decode_exact", dp.data_ptr(), dq.data_ptr(), n, 1.0, 0, d.data_ptr(), st.data_ptr(),
             torch.cuda.current_stream().cuda_stream)
        want = O.reference_delta(p_, q_)
        assert float(d.item()) == want, (n, float(d.item()), want)
        assert int(st[0].item()) == (1 if want < 1.0 else 3)


def test_sdot_order_on_this_host():
    """The box's own numpy: O.sdot_blas (the SkylakeX sdot order the device reproduces) equals x.dot(x) here too."""
    rng = np.random.default_rng(5)
    for n in (33, 64, 1000, 65_537, 1_000_003):
        x = (rng.standard_normal(n) * np.exp(rng.uniform(-3, 3, n))).astype(np.float32)
        assert O.sdot_blas(x, x).view(np.uint32) == np.float32(x.dot(x)).view(np.uint32), n


@pytest.mark.parametrize("side", ["stop", "go_on"])
def test_early_exit_takes_reference_decision(side):
    """eps inside the certified band of an iteration whose reference Δ and f64 Δ differ, just above the reference's Δ
    (it stops there) or just below (it goes on): the device stops for the exact check, fwav_decode_exact decides as
    the reference, and the loop resumes on the device (fwav_decode_from) when it goes on.  Single device and the
    sharded sequence (3 shards) both give the oracle's iteration count and reconstruction bit for bit."""
    from fwav import dist
    idx, s, o, sym, pool = synth_matches(40_000, 6_000, 8, seed=77)
    nr = len(idx)
    base = dict(iterations=40, s_damping=0.5)
    args = (idx, s, o, sym, pool, nr, 8)
    _, _, d64 = O.decode(*args, convergence_eps=0.0, **base)
    _, _, dref = O.decode(*args, convergence_eps=0.0, deltas="reference", **base)
    beta = dist.decode_beta(nr * 8)
    t = next(t for t in range(5, 40) if dref[t] != d64[t])
    eps = dref[t] * (1 + beta / 4) if side == "stop" else dref[t] * (1 - beta / 4)
    assert abs(eps - d64[t]) < beta * d64[t]
    kw = dict(base, convergence_eps=eps)
    ref, it, _ = O.decode(*args, **kw)
    assert (it == t + 1) == (side == "stop")
    rec, ran, deltas = engine.decompress_device(td(idx), td(s), td(o), td(sym), td(pool.reshape(-1)), nr, 8, **kw)
    assert ran == it and bit_equal(rec.cpu().numpy(), ref) and deltas[t] == dref[t]
    outs = _shard_decode(idx, s, o, sym, pool, 8, dist.decode_bounds(nr, 3), kw["iterations"], eps, kw["s_damping"])
    assert bit_equal(np.concatenate([r.cpu().numpy() for r, _, _ in outs]), ref)
    assert all(r_ == it and dl[t] == dref[t] for _, r_, dl in outs)


@pytest.mark.parametrize("side", ["stop", "go_on"])
def test_decode_all_runs_to_the_reference_stop(side):
    """fwav_decode_all (a C-ABI caller that never runs the check loop itself): one call resolves the exact
    check and resumes on its own, with the oracle's iteration count, reconstruction and the reference's Δ at the
    checked iteration — and without a check (default eps) it equals fwav_decode."""
    from fwav import dist
    from fwav._lib import call, size_call
    idx, s, o, sym, pool = synth_matches(40_000, 6_000, 8, seed=77)
    nr = len(idx)
    base = dict(iterations=40, s_damping=0.5)
    args = (idx, s, o, sym, pool, nr, 8)
    _, _, d64 = O.decode(*args, convergence_eps=0.0, **base)
    _, _, dref = O.decode(*args, convergence_eps=0.0, deltas="reference", **base)
    beta = dist.decode_beta(nr * 8)
    t = next(t for t in range(5, 40) if dref[t] != d64[t])
    eps = dref[t] * (1 + beta / 4) if side == "stop" else dref[t] * (1 - beta / 4)
    ref, it, _ = O.decode(*args, convergence_eps=eps, **base)
    dev = torch.device("cuda", 0)
    a = torch.empty(nr * 8, dtype=torch.float32, device=dev)
    b = torch.empty_like(a)
    deltas = torch.zeros(40, dtype=torch.float64, device=dev)
    state = torch.zeros(4, dtype=torch.int32, device=dev)
    wsn = size_call("fwav_decode_all_workspace_size", nr, 8, 40)
    ws = torch.empty(wsn, dtype=torch.uint8, device=dev)
    ti, ts, to, tsym, tp = td(idx), td(s), td(o), td(sym), td(pool.reshape(-1))
    call("fwav_decode_all", ti.data_ptr(), ts.data_ptr(), to.data_ptr(), tsym.data_ptr(), nr, 8, tp.data_ptr(),
         len(pool), 40, eps, 16.0, 0.5, a.data_ptr(), b.data_ptr(), deltas.data_ptr(), state.data_ptr(),
         ws.data_ptr(), wsn, torch.cuda.current_stream().cuda_stream)
    st = state.cpu().numpy()
    out = (b if st[2] == 1 else a).cpu().numpy()
    # "go_on": the reference goes on at iteration t + 1 (the check) and stops later, or runs every iteration
    assert st[1] == it and st[0] == (1 if it < 40 else 0), (st, it)
    assert (it == t + 1) == (side == "stop")
    assert bit_equal(out, ref) and deltas.cpu().numpy()[t] == dref[t]
