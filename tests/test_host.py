"""Host-side product code: .fwav container, WAV I/O, match records, CLI surface (no GPU)."""
import os
import struct

import numpy as np
import pytest

from golden_util import load


def _ml(g, K):
    from fwav.matches import MatchList
    return MatchList(g[f"m_idx_{K}"], g[f"m_s_{K}"], g[f"m_o_{K}"], g[f"m_sym_{K}"], g[f"m_err_{K}"])


@pytest.mark.parametrize("case,K", [("tone", 32), ("sweep", 64), ("ragged", 16)])
def test_save_compressed_bytes_match_reference(tmp_path, case, K):
    from fwav.fwavio import save_compressed
    g = load(case)
    p = g["p"]
    fp = tmp_path / "x.fwav"
    save_compressed(str(fp), _ml(g, K), g["pool"], p["rs"], p["framerate"], p["sampwidth"], p["tile"], p["step"],
                    p["thr"], p["original_len"])
    assert fp.read_bytes() == g[f"fwav_{K}"].tobytes()
    # a plain list of tuples gives the same bytes
    fp2 = tmp_path / "y.fwav"
    save_compressed(str(fp2), list(_ml(g, K)), g["pool"], p["rs"], p["framerate"], p["sampwidth"], p["tile"],
                    p["step"], p["thr"], p["original_len"])
    assert fp2.read_bytes() == fp.read_bytes()


def test_load_compressed_roundtrip_and_errors(tmp_path):
    from fwav.fwavio import load_compressed
    g = load("sweep")
    fp = tmp_path / "s.fwav"
    fp.write_bytes(g["fwav_32"].tobytes())
    m, dom, nr, rs, fr, sw, tile, step, thr, orig = load_compressed(str(fp))
    p = g["p"]
    assert (nr, rs, fr, sw, tile, step, orig) == (p["n_ranges"], p["rs"], 16000, 2, 512, 1, p["original_len"])
    assert np.float32(thr) == np.float32(p["thr"])
    assert np.array_equal(dom, g["pool"])
    assert m[5] == (int(g["m_idx_32"][5]), float(g["m_s_32"][5]), float(g["m_o_32"][5]), int(g["m_sym_32"][5]),
                    float(g["m_err_32"][5]))
    assert all(isinstance(v, t) for v, t in zip(m[0], (int, float, float, int, float)))
    raw = bytearray(g["fwav_32"].tobytes())
    bad = tmp_path / "bad.fwav"
    bad.write_bytes(b"XXXX" + raw[4:])
    with pytest.raises(ValueError, match="Not a FWAV"):
        load_compressed(str(bad))
    bad.write_bytes(raw[:4] + b"\x02" + raw[5:])
    with pytest.raises(ValueError, match="Unsupported FWAV version"):
        load_compressed(str(bad))
    flip = bytearray(raw)
    flip[100] ^= 1
    bad.write_bytes(bytes(flip))
    with pytest.raises(ValueError, match="Checksum mismatch"):
        load_compressed(str(bad))
    load_compressed(str(bad), verify_checksum=False)
    # a header whose counts promise more bytes than the file holds (truncated or hostile): no allocation from the
    # counts; a short payload fails its checksum first, as in the reference, which hashes whatever follows the header
    from fwav.fwavio import HEADER_FMT
    fields = list(struct.unpack(HEADER_FMT, raw[:struct.calcsize(HEADER_FMT)]))
    fields[9] = 0xFFFFFFFF  # n_domains: 4 Gi domain rows (32 GiB at range_size 2)
    huge = struct.pack(HEADER_FMT, *fields) + raw[struct.calcsize(HEADER_FMT):]
    bad.write_bytes(huge)  # (the checksum covers the payload only, so it still matches)
    for verify in (True, False):
        with pytest.raises(ValueError, match="truncated FWAV file"):
            load_compressed(str(bad), verify_checksum=verify)
    bad.write_bytes(raw[:-5])
    with pytest.raises(ValueError, match="Checksum mismatch"):
        load_compressed(str(bad))
    with pytest.raises(ValueError, match="truncated FWAV file"):
        load_compressed(str(bad), verify_checksum=False)


def test_empty_fwav_cannot_be_loaded(tmp_path):
    """The reference writes n_domains=0 files that its own loader rejects (np.vstack([]), fractal.py:1372)."""
    from fwav.fwavio import load_compressed, save_compressed
    fp = tmp_path / "e.fwav"
    save_compressed(str(fp), [], np.zeros((0, 8), np.float32), 8, 44100, 4, 2048, 2, 1e-4, 100)
    assert os.path.getsize(fp) == 66
    with pytest.raises(ValueError):
        load_compressed(str(fp))


@pytest.mark.parametrize("sw", [1, 2, 3, 4])
def test_wav_roundtrip(tmp_path, sw):
    from fwav.fwavio import read_wav_mono, write_wav
    rng = np.random.default_rng(sw)
    if sw == 4:
        x = rng.uniform(-1, 1, 999).astype(np.float32)
    else:
        lim = {1: 127, 2: 32767, 3: 2 ** 23 - 1}[sw]
        x = rng.integers(-lim, lim, 999).astype(np.float32)
    fp = str(tmp_path / f"a{sw}.wav")
    write_wav(fp, x, 22050, sw)
    y, fr, sw2 = read_wav_mono(fp)
    assert fr == 22050 and sw2 == sw and y.dtype == np.float32
    assert np.array_equal(y, x)


def test_header_layout():
    from fwav import fwavio
    assert fwavio.HEADER_SIZE == 34
    assert struct.calcsize("<iffBf") == 17 == fwavio.MATCH_DTYPE.itemsize


def test_matchlist_sequence():
    from fwav.matches import MatchList, as_match_arrays
    m = MatchList([1, 2], [0.5, -1.0], [0.25, 3.0], [0, 1], [np.inf, 2.0])
    assert len(m) == 2 and m[1] == (2, -1.0, 3.0, 1, 2.0)
    assert list(m) == [m[0], m[1]] and m == [m[0], m[1]]
    a = as_match_arrays([(3, 1.5, 2.5, 1, 0.5)])
    assert a[0].dtype == np.int32 and a[3].dtype == np.uint8 and a[0][0] == 3


def test_geometry_matches_reference():
    from fwav.engine import geometry
    for tile, exp in [(128, (4, 1)), (512, (4, 1)), (1024, (4, 1)), (2048, (8, 2)), (4096, (16, 4)),
                      (65535, (255, 63))]:
        assert geometry(tile) == exp


def test_cli_parser_help(capsys):
    from fwav.cli import main
    assert main([]) is None
    assert "compress" in capsys.readouterr().out
    with pytest.raises(SystemExit):
        main(["compress", "in.wav"])  # OUTPUT required unless --batch


def test_reflect_index_formula():
    """k_form_ranges / k_frame_energy use the np.pad reflect index p → q (period 2(n−1)); checked here on CPU."""
    def reflect_idx(p, n):
        if p < n:
            return p
        if n == 1:
            return 0
        per = 2 * (n - 1)
        q = p % per
        return q if q < n else per - q
    for n in (1, 2, 3, 5, 17):
        x = np.arange(n)
        for pad in range(0, 3 * n + 2):
            ref = np.pad(x, (0, pad), mode="reflect") if n > 1 or pad == 0 else np.pad(x, (0, pad), mode="edge")
            got = np.array([x[reflect_idx(p, n)] for p in range(n + pad)])
            assert np.array_equal(ref, got), (n, pad)


def test_product_path_fails_loudly_without_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a device is present")
    from fwav import api
    from fwav._lib import FwavError
    with pytest.raises(FwavError):
        api.compress_audio(np.zeros(5000, np.float32), 44100, 4, tile_size=1024)


def test_sub_block_slices():
    """fwav.engine's sliced search (large tables): slices cover the active list exactly once, in order, the last one
    about half the others; the slice count follows the table size and the query count."""
    from fwav import engine
    for m, n in ((2_700_000, 8), (1_653_750, 4), (10, 3), (5, 5), (3, 7), (1, 1)):
        b = engine._slice_bounds(m, n)
        assert b[0][0] == 0 and b[-1][1] == m and all(b[i][1] == b[i + 1][0] for i in range(len(b) - 1))
        assert all(hi > lo for lo, hi in b)
        if m >= 100 * n and n > 1:
            sizes = [hi - lo for lo, hi in b]
            assert abs(sizes[-1] * 2 - sizes[0]) <= 2 and len(set(sizes[:-1])) <= 2
    assert engine._tie_sub_blocks(330_750, 1_321_977) == 1        # cfg2: table below 4 Mi domains
    assert engine._tie_sub_blocks(1_653_750, 6_613_977) == 4      # cfg3
    assert engine._tie_sub_blocks(2_700_000, 86_398_977) == 6     # one rank's eighth of cfg4
    assert engine._tie_sub_blocks(21_600_000, 86_398_977) == 8    # all of cfg4 on one GPU
    assert engine._tie_sub_blocks(100_000, 86_398_977) == 1
