"""The C ABI on its own: numpy in/out through ctypes + libamdhip64, no torch tensors (INTEGRATION.md binding).

``fwav.hipctypes.compress`` / ``decompress`` drive the whole device sequence (voiced ranges → silent test → pool and
embeddings → prune → search → affine → tie check → numpy's ranking of the listed rows → fix-up; the decode loop) with
HIP buffers alone, in a child process that must never import torch; every match tuple and every decoded sample is
bit-exact with the reference's goldens (cpu_worker fractal.py:556-632, _process_gpu_batch :757-870,
decompress_audio :1378-1473)."""
import os
import subprocess
import sys

import numpy as np
import pytest

from golden_util import bit_equal, load

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


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
    assert bit_equal(emb, g["emb"])


_CHILD = r"""
import sys
sys.path[:0] = [{tests!r}, {pkg!r}]
import numpy as np
from golden_util import bit_equal, load
from fwav import hipctypes as H

for case, K in (("tone", 32), ("speech4096", 64), ("ragged", 16), ("tiny", 8), ("noise2048", 64)):
    g = load(case)
    p = g["p"]
    r = H.compress(g["signal"], p["tile"], K, energy_thresh=p["thr"])
    assert r is not None and r["n_ranges"] == p["n_ranges"] and r["n_domains"] == p["n_domains"], case
    assert bit_equal(r["pool"], g["pool"]) and bit_equal(r["emb"], g["emb"]), case
    for nm in ("idx", "s", "o", "sym", "err"):
        assert bit_equal(r[nm], g[f"m_{{nm}}_{{K}}"]), (case, nm)
    args = [g[f"m_{{nm}}_{{K}}"] for nm in ("idx", "s", "o", "sym")] + [g["pool"], p["n_ranges"], p["rs"]]
    rec, it, _ = H.decompress(*args, original_len=p["original_len"])
    assert bit_equal(rec, g[f"dec_{{K}}"]) and it == int(g[f"dec_iters_{{K}}"]), case
    rec, it, _ = H.decompress(*args, iterations=50, convergence_eps=0.0, original_len=p["original_len"])
    assert bit_equal(rec, g[f"dec50_{{K}}"]) and it == 50, case
    print(f"{{case}} K={{K}}: {{r['n_ranges']}} ranges, {{r['n_ties']}} tied rows, {{r['n_resolved']}} ranked by numpy; "
          "tuples and decodes bit-exact")
# the reference's empty / error cases
assert H.compress(np.zeros(4000, np.float32), 2048, 64) is None
assert H.compress(np.ones(100, np.float32), 2048, 64) is None
try:
    H.compress(np.ones(2448, np.float32) * 0.5, 2048, 64)
    raise SystemExit("quirk Q9 not raised")
except ValueError as e:
    assert "mmap length" in str(e)
assert "torch" not in sys.modules, "the torch-free binding imported torch"
print("TORCH_FREE_OK")
"""


def test_compress_decompress_ctypes_only_bitexact():
    """compress_audio + decompress_audio through the C ABI with numpy and HIP buffers only (the tone case has exact
    score ties ranked by numpy's own calls)."""
    code = _CHILD.format(tests=os.path.join(ROOT, "tests"), pkg=os.path.join(ROOT, "audio-compression_amd"))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    print(out.stdout[-3000:], out.stderr[-3000:])
    assert out.returncode == 0 and "TORCH_FREE_OK" in out.stdout
    assert "tone K=32" in out.stdout
