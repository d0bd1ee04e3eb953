"""GPU decode (fwav_decode.hip) against the oracle's decompress_audio restatement (fractal.py:1378-1473).

The iteration-resident kernel runs up to 64 iterations per launch with each range's reconstruction in registers and
recomputes the stopping chunk, so these cases cover: a stop inside the second chunk, forced runs across
chunk boundaries (64, 65, 130 iterations), every range_size bucket (exact 4/8/16/32, guarded 5/12/20/31) and the
streaming path (range_size > 32), sentinel −1 indices and constant tiles (‖T − mean T‖² = 0).  Bar: recon bit-exact,
the same iteration count, Δ within 1e-12 relative (f64 sums, different order from numpy's).
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
    assert ran == it, (ran, it)
    assert bit_equal(rec.cpu().numpy(), ref)
    np.testing.assert_allclose(deltas, rdel, rtol=1e-12, atol=0)
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
    all-reduce of fwav.dist.decompress_sharded does."""
    from fwav import dist
    nr = len(idx)
    decs = [dist.ShardDecoder(td(idx[a:b]), td(s[a:b]), td(o[a:b]), td(sym[a:b]), td(pool.reshape(-1)), a, nr, rs,
                              iterations, eps, 16.0, s_damping) for a, b in bounds]
    for c in range(decs[0].n_chunks):
        for d in decs:
            d.run(c)
        tot = sum(d.partials_prefix() for d in decs)
        for d in decs:
            d.partials_prefix().copy_(tot)
            d.reduce(c)
    outs = [d.finish() for d in decs]
    return outs


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
