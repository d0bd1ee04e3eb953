"""GPU: the fractal-compatible API surface — reference edge cases, sentinels, shards, CLI end to end."""
import json
import os

import numpy as np
import pytest

from golden_util import GOLDEN, bit_equal

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def test_reference_edge_cases():
    import fractal
    from fwav import synth
    edges = json.load(open(os.path.join(GOLDEN, "edges.json")))
    r = fractal.compress_audio(synth.noise(0.01, 44100, seed=5), 44100, 4, tile_size=2048)
    assert len(r[0]) == edges["short"]["n_matches"] and list(r[1].shape) == edges["short"]["pool_shape"]
    assert [int(r[2]), int(r[3]), int(r[4]), int(r[5]), float(r[6]), int(r[7])] == edges["short"]["rest"]
    r = fractal.compress_audio(np.zeros(5000, np.float32), 44100, 4, tile_size=1024)
    assert len(r[0]) == 0 and list(r[1].shape) == edges["silent"]["pool_shape"]
    assert [int(r[2]), int(r[3]), int(r[4]), int(r[5]), float(r[6]), int(r[7])] == edges["silent"]["rest"]
    with pytest.raises(ValueError, match=edges["q9"]["msg"]):
        fractal.compress_audio(synth.noise(1.0, 44100)[:2448], 44100, 4, tile_size=2048)


def test_decode_sentinels_match_oracle():
    from fwav.api import decompress_audio
    from oracle import fractal_oracle as O
    rng = np.random.default_rng(4)
    nd, rs, nr = 300, 8, 200
    pool = rng.normal(size=(nd, rs)).astype(np.float32)
    pool[7] = 1.0  # constant tile: denominator 0 → stored s used
    idx = rng.integers(-1, nd, nr).astype(np.int32)
    idx[::17] = 7
    s = rng.normal(size=nr).astype(np.float32) * 3
    o = rng.normal(size=nr).astype(np.float32)
    sym = rng.integers(0, 2, nr).astype(np.uint8)
    m = list(zip(idx.tolist(), s.tolist(), o.tolist(), sym.tolist(), [0.0] * nr))
    for kw in (dict(), dict(iterations=20, convergence_eps=0.0), dict(iterations=9, convergence_eps=0.0, s_damping=0.5),
               dict(iterations=5, s_clip=0.75)):
        d, info = decompress_audio(m, pool, nr, rs, original_len=nr * rs - 3, return_info=True, **kw)
        ref, it, _ = O.decode(idx, s, o, sym, pool, nr, rs, original_len=nr * rs - 3, **kw)
        assert bit_equal(d, ref) and info["iterations"] == it


def test_shards_concatenate_to_full_run():
    from fwav import engine, synth
    sig = torch.from_numpy(synth.speech_like(3.0, 44100, seed=9, floor=False)).cuda()
    full = engine.compress_device(sig, 2048, 32, keep_intermediates=True)
    nr = full.n_ranges
    cuts = [0, 1000, 1001, 4000, nr]
    parts = [engine.compress_device(sig, 2048, 32, shard=(a, b)) for a, b in zip(cuts[:-1], cuts[1:])]
    torch.cuda.synchronize()
    for f in ("idx", "s", "o", "sym", "err"):
        cat = np.concatenate([getattr(p, f).cpu().numpy() for p in parts])
        assert bit_equal(cat, getattr(full, f).cpu().numpy()), f


def test_cli_roundtrip(tmp_path):
    from fwav import synth
    from fwav.cli import main
    from fwav.fwavio import write_wav
    wav = tmp_path / "a.wav"
    write_wav(str(wav), synth.noise(0.5, 22050, seed=3), 22050, 4)
    out = tmp_path / "out"
    r = main(["compress", str(wav), str(out), "--tile", "1024"])
    assert "error" not in r and os.path.exists(out / "a.wav.fwav")
    r = main(["decompress", str(out / "a.wav.fwav"), "--out", str(tmp_path / "rec")])
    assert "error" not in r and os.path.exists(tmp_path / "rec" / "a.wav.fwav_recon.wav")


def test_cli_batch_one_process_per_gpu(tmp_path):
    """Batch mode (fractal.py:1581-1610, 1625-1655): one worker process per visible GPU (at most --workers), files in
    input order; every file compressed and decompressed, identical to the single-file command's outputs, metrics
    written, existing outputs skipped on a rerun."""
    import json
    from fwav import synth
    from fwav.cli import main, _gpu_count
    from fwav.fwavio import write_wav
    src = tmp_path / "wav"
    src.mkdir()
    for i in range(3):
        write_wav(str(src / f"f{i}.wav"), synth.noise(0.3, 22050, seed=i), 22050, 4)
    out = tmp_path / "out"
    res = main(["compress", str(src), "--batch", "--out", str(out), "--tile", "1024", "--workers", "8"])
    assert len(res) == 3 and not any("error" in r for r in res)
    assert [os.path.basename(r["input"]) for r in res] == [f for f in os.listdir(src) if f.endswith(".wav")]
    assert json.load(open(out / "compression_metrics.json")) == res
    one = tmp_path / "one"
    main(["compress", str(src / "f1.wav"), str(one), "--tile", "1024"])
    # the batch job's OUTPUT argument is itself used as a directory (quirk Q8 applies to batch jobs too)
    assert (one / "f1.wav.fwav").read_bytes() == (out / "f1.wav.fwav" / "f1.wav.fwav").read_bytes()
    assert main(["compress", str(src), "--batch", "--out", str(out), "--tile", "1024"]) is None  # all exist
    fw = tmp_path / "fw"
    fw.mkdir()
    for i in range(3):
        (fw / f"f{i}.wav.fwav").write_bytes((out / f"f{i}.wav.fwav" / f"f{i}.wav.fwav").read_bytes())
    dres = main(["decompress", str(fw), "--batch", "--out", str(tmp_path / "rec")])
    assert len(dres) == 3 and not any("error" in r for r in dres)
    assert _gpu_count() >= 1


@pytest.mark.parametrize("case", ["tone", "sweep"])
def test_cli_outputs_match_reference(tmp_path, case):
    """`fractal.py compress IN.wav OUT --tile T` then `decompress` (fractal.py:1491-1546, quirk Q8 directories):
    the .fwav the CLI writes is the reference's file byte for byte, and decompressing the reference's own .fwav
    through the CLI writes exactly the reference's reconstruction as 16-bit PCM."""
    from fwav.cli import main
    from fwav.fwavio import read_wav_mono, write_wav
    from golden_util import load
    g = load(case)
    p = g["p"]
    wav = tmp_path / f"{case}.wav"
    write_wav(str(wav), g["signal"], p["framerate"], p["sampwidth"])
    sig, fr, sw = read_wav_mono(str(wav))
    assert bit_equal(sig, g["signal"]) and (fr, sw) == (p["framerate"], p["sampwidth"])
    r = main(["compress", str(wav), str(tmp_path / "out"), "--tile", str(p["tile"])])
    assert "error" not in r, r
    mine = np.frombuffer((tmp_path / "out" / f"{case}.wav.fwav").read_bytes(), np.uint8)
    ref = g["fwav_32"]  # the CLI uses the module-global K = 32 (quirk Q2)
    assert np.array_equal(mine, ref)
    # decompress the reference's .fwav with the CLI defaults (--iter 8 --eps 1e-3)
    fw = tmp_path / f"{case}_ref.fwav"
    fw.write_bytes(ref.tobytes())
    r = main(["decompress", str(fw), "--out", str(tmp_path / "rec")])
    assert "error" not in r, r
    out, fr2, sw2 = read_wav_mono(str(tmp_path / "rec" / f"{case}_ref.fwav_recon.wav"))
    expect = g["dec_32"].clip(-32768, 32767).astype(np.int16).astype(np.float32)  # write_wav, sampwidth 2
    assert (fr2, sw2) == (p["framerate"], 2) and bit_equal(out, expect)
