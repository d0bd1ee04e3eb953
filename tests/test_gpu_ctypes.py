"""The C ABI on its own: numpy in/out through ctypes + libamdhip64, no torch tensors (INTEGRATION.md binding)."""
import numpy as np
import pytest

from golden_util import bit_equal, load

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case,k", [("noise2048", 64), ("sweep", 32), ("speech4096", 64)])
def test_affine_ctypes_only_bitexact(case, k):
    from fwav import hipctypes

    g = load(case)
    if f"cand_{k}" not in g:
        pytest.skip(f"no K={k} golden for {case}")
    idx, s, o, sym, err = hipctypes.affine_batch(g["ranges"], g[f"cand_{k}"], g["pool"])
    assert np.array_equal(idx, g[f"m_idx_{k}"])
    assert np.array_equal(sym, g[f"m_sym_{k}"])
    assert bit_equal(s, g[f"m_s_{k}"])
    assert bit_equal(o, g[f"m_o_{k}"])
    assert bit_equal(err, g[f"m_err_{k}"])


def test_pool_embed_ctypes_only():
    from fwav import hipctypes

    g = load("noise2048")
    p = g["p"]
    pool, emb = hipctypes.pool_embed(g["signal"], p["tile"], p["rs"], p["step"])
    assert bit_equal(pool, g["pool"])
    assert np.max(np.abs(emb - g["emb"])) <= 1e-6
