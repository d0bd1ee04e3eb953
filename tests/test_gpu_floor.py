"""The fp16 search's speculative floor (fwav_topk.hip, FloorCtl): a first pass whose band limits start at a floor
guessed from pilot queries, the queries it may have cut searched again without it.  Whatever the floor, the candidates
and every match tuple must equal the all-f32 search's: a floor below every score (nothing cut), floors inside the
range of the K-th scores (some queries cut), one above every score (every query cut), and the pilots' own floor; the
same floor for the second pass too, so that its cuts take the floor-free third pass — under
each first-pass mode and geometry, with split plans, and on a signal whose bands overflow."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from fwav import engine, synth  # noqa: E402
from fwav._lib import call, debug_library  # noqa: E402


def td(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(torch.device("cuda", 0))


def _run(sig, tile, K, search):
    r = engine.compress_device(td(sig), tile, K, energy_thresh=1e-4, keep_intermediates=True, search=search,
                               tie_order="numpy_sets")
    torch.cuda.synchronize()
    return r.cand.cpu().numpy().reshape(-1, K), r


def _kth_scores(r, cand):
    """The K-th score of every searched query (the active list: the energy prune's survivors), in f64."""
    emb = r.emb.cpu().numpy().reshape(-1, 16).astype(np.float64)
    q = r.active[:int(r.n_active.item())].cpu().numpy().astype(np.int64)
    q = q[cand[q, -1] >= 0]
    return (emb[q] * emb[cand[q, -1]]).sum(1)


def _periodic(n=24000, period=96):
    t = np.arange(n)
    return np.round(8000 * np.sin(2 * np.pi * t / period) + 3000 * np.sin(2 * np.pi * 3 * t / period)
                    ).astype(np.float32)


SIGNALS = {
    "noise": (lambda: synth.noise(6.0, 44100, seed=11), 2048, 64),
    "speech": (lambda: synth.speech_like(6.0, 44100, seed=5), 4096, 17),
    "periodic": (_periodic, 1024, 32),
}


def _check(sig, tile, K, floors, ref):
    b, rb = ref
    for mode, value in floors:
        with debug_library():
            call("fwav_debug_topk_floor", mode, value)
            a, ra = _run(sig, tile, K, "f16")
        assert np.array_equal(a, b), (mode, value)
        for x, y in ((ra.idx, rb.idx), (ra.s, rb.s), (ra.o, rb.o), (ra.sym, rb.sym), (ra.err, rb.err)):
            assert np.array_equal(x.cpu().numpy().view(np.uint8), y.cpu().numpy().view(np.uint8)), (mode, value)


@pytest.mark.parametrize("gen", list(SIGNALS))
def test_floor_any_value_equals_f32(gen):
    mk, tile, K = SIGNALS[gen]
    sig = mk()
    ref = _run(sig, tile, K, "f32")
    kth = _kth_scores(ref[1], ref[0])
    assert len(kth) > 1000
    qs = [float(np.quantile(kth, p)) for p in (0.01, 0.3, 0.7)]
    # mode 3: the second pass at the same floor, so the queries it cuts go on to the floor-free third pass
    floors = [(0, 0.0), (1, -10.0), *[(1, v) for v in qs], (1, float(kth.max()) + 0.01), (1, 10.0), (2, 0.0),
              (3, qs[0]), (3, qs[1]), (3, 10.0)]
    _check(sig, tile, K, floors, ref)


@pytest.fixture(params=[(0, 0), (1, 0), (0, 1), (1, 1), (0, 2), (1, 2), (0, 3), (1, 3)],
                ids=["s16-base", "hl-base", "s16-wide", "hl-wide", "s16-cent", "hl-cent", "s16-centw", "hl-centw"])
def geometry(request):
    mode, wide = request.param
    with debug_library():
        call("fwav_debug_topk_mode", mode)
        call("fwav_debug_topk_geometry", wide)
        yield mode, wide


def test_floor_every_geometry(geometry):
    """Inside one debug_library block (the geometry fixture's): the floor knob on top of each first-pass mode and
    geometry, a floor at the median K-th score (half the queries cut) and the pilots' floor."""
    mk, tile, K = SIGNALS["noise"]
    sig = mk()
    b, rb = _run(sig, tile, K, "f32")
    kth = _kth_scores(rb, b)
    for mode, value in ((1, float(np.median(kth))), (2, 0.0), (3, float(np.quantile(kth, 0.05)))):
        call("fwav_debug_topk_floor", mode, value)
        a, _ = _run(sig, tile, K, "f16")
        assert np.array_equal(a, b), (geometry, mode, value)
    call("fwav_debug_topk_floor", -1, 0.0)


@pytest.mark.parametrize("plan", [(1 << 20, 2), (1 << 20, 8), (10, 3), (1 << 20, -1)])
def test_floor_split_plans(plan):
    """First-pass plans with table pieces (k_merge_pieces takes the floor decision) and query halves."""
    mk, tile, K = SIGNALS["noise"]
    sig = mk()
    b, rb = _run(sig, tile, K, "f32")
    v = float(np.quantile(_kth_scores(rb, b), 0.5))
    with debug_library():
        call("fwav_debug_topk_plan", *plan)
        call("fwav_debug_topk_floor", 1, v)
        a, _ = _run(sig, tile, K, "f16")
    assert np.array_equal(a, b)
