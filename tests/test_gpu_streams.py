"""Consecutive compress calls alternating over two HIP streams (bench.py --streams 2, the N > 1 default): every call's
outputs equal one synchronous call's, with numpy-order tie rows deferred and applied on each call's own stream, and
with the search's speculative floor in play (a signal of more than 65,536 ranges)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from fwav import engine, synth  # noqa: E402


@pytest.mark.parametrize("gen,seconds,tile", [("speech", 8.0, 2048), ("noise", 14.0, 2048)])
def test_two_streams_equal_one_call(gen, seconds, tile):
    dev = torch.device("cuda", 0)
    mk = synth.speech_like if gen == "speech" else synth.noise
    sig = torch.from_numpy(mk(seconds, 44100, seed=7)).to(dev)
    ref = engine.compress_device(sig, tile, 64, energy_thresh=1e-4)
    torch.cuda.synchronize()
    want = [t.cpu().numpy() for t in (ref.idx, ref.s, ref.o, ref.sym, ref.err)]
    streams = [torch.cuda.current_stream(dev), torch.cuda.Stream(dev)]
    calls = []
    for i in range(6):
        with torch.cuda.stream(streams[i % 2]):
            calls.append(engine.compress_device(sig, tile, 64, energy_thresh=1e-4, defer_ties=True))
    for r in calls:
        r.wait()
    torch.cuda.synchronize()
    for r in calls:
        got = [t.cpu().numpy() for t in (r.idx, r.s, r.o, r.sym, r.err)]
        for a, b in zip(got, want):
            assert np.array_equal(a.view(np.uint8), b.view(np.uint8))
