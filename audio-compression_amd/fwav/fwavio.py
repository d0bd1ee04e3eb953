"""WAV I/O and the ``.fwav`` container (byte-identical to the reference).

Reference: ``read_wav_mono`` fractal.py:81-113, ``write_wav`` :116-137, ``save_compressed`` :1278-1322,
``load_compressed`` :1325-1375.  The reference writes/reads one domain row and one match at a time
(86 M ``f.read`` calls at cfg4); here both sections move as single buffers with a streaming SHA-256 over
exactly the same bytes (domains ‖ matches; the header is not hashed, as in the reference).

Layout (little-endian, packed):
  'FWAV' | u8 version=1 | u32 range_size | u32 framerate | u8 sampwidth | u16 tile_size | u16 domain_step |
  f32 energy_threshold | u32 n_ranges | u32 n_domains | u32 original_len | 32 B SHA-256 |
  f32[n_domains, range_size] | n_ranges × '<iffBf' (domain_idx, s, o, sym, err)
"""
from __future__ import annotations

import hashlib
import os
import struct
import wave
from concurrent.futures import ThreadPoolExecutor

import numpy as np

from .matches import MATCH_DTYPE, MatchList, as_match_arrays

FWAV_VERSION = 1
HEADER_FMT = "<4sBIIBHHfIII"
HEADER_SIZE = struct.calcsize(HEADER_FMT)
_CHUNK = 1 << 24


def read_wav_mono(path, mmap=False):
    """fractal.py:81-113: int PCM stays in integer units (as float32), multichannel → mean."""
    with wave.open(path, "rb") as w:
        nchan = w.getnchannels()
        sampwidth = w.getsampwidth()
        framerate = w.getframerate()
        nframes = w.getnframes()
        comptype = w.getcomptype()
        if comptype != "NONE":
            raise ValueError(f"Unsupported WAV compression type: {comptype}")
        raw = w.readframes(nframes)
    if sampwidth == 1:
        data = np.frombuffer(raw, dtype=np.uint8).astype(np.int16) - 128
    elif sampwidth == 2:
        data = np.frombuffer(raw, dtype=np.int16)
    elif sampwidth == 3:
        b = np.frombuffer(raw, dtype=np.uint8).reshape(-1, 3).astype(np.int32)
        data = b[:, 0] | (b[:, 1] << 8) | (b[:, 2] << 16)
        data = data - ((data & 0x800000) << 1)
    elif sampwidth == 4:
        data = np.frombuffer(raw, dtype=np.float32)
    else:
        raise ValueError(f"Unsupported sample width: {sampwidth}")
    if nchan > 1:
        data = data.reshape(-1, nchan).mean(axis=1)
    return data.astype(np.float32), framerate, sampwidth


def write_wav(path, data, framerate, sampwidth):
    """fractal.py:116-137."""
    data = np.asarray(data)
    if sampwidth == 1:
        out = (data + 128).clip(0, 255).astype(np.uint8)
    elif sampwidth == 2:
        out = data.clip(-32768, 32767).astype(np.int16)
    elif sampwidth == 3:
        d32 = data.clip(-2 ** 23, 2 ** 23 - 1).astype(np.int32)
        out = np.column_stack([(d32 & 0xFF).astype(np.uint8), ((d32 >> 8) & 0xFF).astype(np.uint8),
                               ((d32 >> 16) & 0xFF).astype(np.uint8)]).flatten()
    elif sampwidth == 4:
        out = data.astype(np.float32)
    else:
        raise ValueError(f"Unsupported sample width: {sampwidth}")
    with wave.open(path, "wb") as w:
        w.setnchannels(1)
        w.setsampwidth(sampwidth)
        w.setframerate(framerate)
        w.writeframes(out.tobytes())


def _match_records(matches) -> np.ndarray:
    idx, s, o, sym, err = as_match_arrays(matches)
    rec = np.empty(len(idx), MATCH_DTYPE)
    rec["idx"], rec["s"], rec["o"], rec["sym"], rec["err"] = idx, s, o, sym, err
    return rec


class _Hasher:
    """SHA-256 of a byte stream on a worker thread (hashlib releases the GIL on large updates), so that hashing
    overlaps the file reads or writes of the same chunks."""

    def __init__(self):
        self.sha = hashlib.sha256()
        self.pool = ThreadPoolExecutor(1)
        self.pending = None

    def update(self, buf):
        if self.pending is not None:
            self.pending.result()
        self.pending = self.pool.submit(self.sha.update, buf)

    def digest(self) -> bytes:
        if self.pending is not None:
            self.pending.result()
        self.pool.shutdown()
        return self.sha.digest()


def save_compressed(filepath, matches, domains_array, range_size, framerate, sampwidth, tile_size, domain_step,
                    energy_threshold, original_len):
    """fractal.py:1278-1322 — same bytes: the domain rows and the packed match records written as two bulk
    buffers in chunks, each chunk hashed on a worker thread while the next one is written."""
    rec = _match_records(matches)
    dom = np.ascontiguousarray(np.asarray(domains_array), dtype="<f4")
    n_domains = len(dom)
    hdr = struct.pack(HEADER_FMT, b"FWAV", FWAV_VERSION, range_size, framerate, sampwidth, tile_size, domain_step,
                      energy_threshold, len(rec), n_domains, original_len)
    sha = _Hasher()
    dbytes = memoryview(dom.reshape(-1).view(np.uint8))
    mbytes = memoryview(rec.view(np.uint8))
    with open(filepath, "wb") as f:
        f.write(hdr)
        f.write(b"\0" * 32)
        for buf in (dbytes, mbytes):
            for i in range(0, len(buf), _CHUNK):
                piece = buf[i:i + _CHUNK]
                sha.update(piece)
                f.write(piece)
        f.seek(HEADER_SIZE)
        f.write(sha.digest())


def _read_into(f, arr: np.ndarray, sha: "_Hasher | None") -> int:
    """Fill arr's bytes from f in chunks (no intermediate bytes objects); returns the bytes read."""
    buf = memoryview(arr.reshape(-1).view(np.uint8))
    got = 0
    while got < len(buf):
        n = f.readinto(buf[got:got + _CHUNK])
        if not n:
            break
        if sha is not None:
            sha.update(buf[got:got + n])
        got += n
    return got


def load_compressed(filepath, verify_checksum=True):
    """fractal.py:1325-1375 — returns (matches, domains, n_ranges, range_size, framerate, sampwidth, tile_size,
    domain_step, energy_threshold, original_len); ``matches`` is a :class:`MatchList` (a sequence of the
    reference's ``(int, float, float, int, float)`` tuples backed by arrays).  Both sections are read straight into
    their final arrays (the domain rows, the packed records whose fields the MatchList views), hashed on a worker
    thread as they arrive."""
    with open(filepath, "rb") as f:
        if f.read(4) != b"FWAV":
            raise ValueError("Not a FWAV file")
        version = struct.unpack("<B", f.read(1))[0]
        if version != FWAV_VERSION:
            raise ValueError(f"Unsupported FWAV version: {version}")
        f.seek(0)
        (_, _, range_size, framerate, sampwidth, tile_size, domain_step, energy_threshold, n_ranges, n_domains,
         original_len) = struct.unpack(HEADER_FMT, f.read(HEADER_SIZE))
        stored = f.read(32)
        sha = _Hasher() if verify_checksum else None
        need = 4 * range_size * n_domains + MATCH_DTYPE.itemsize * n_ranges
        if os.fstat(f.fileno()).st_size - f.tell() < need:
            # a truncated (or hostile) header: no allocation from its counts; the checksum still decides first, as
            # in the reference, which hashes whatever follows the header
            if sha is not None:
                while True:
                    piece = f.read(_CHUNK)
                    if not piece:
                        break
                    sha.update(piece)
                if sha.digest() != stored:
                    raise ValueError("Checksum mismatch — file may be corrupted")
            raise ValueError("truncated FWAV file")
        domains = np.empty((n_domains, range_size), np.float32)
        rec = np.empty(n_ranges, MATCH_DTYPE)
        got_d = _read_into(f, domains, sha)
        got_m = _read_into(f, rec, sha)
    if sha is not None and sha.digest() != stored:
        raise ValueError("Checksum mismatch — file may be corrupted")
    if n_domains == 0:
        raise ValueError("need at least one array to concatenate")  # np.vstack([]) in the reference (:1372)
    if got_d != domains.nbytes or got_m != rec.nbytes:
        raise ValueError("truncated FWAV file")
    matches = MatchList(rec["idx"], rec["s"], rec["o"], rec["sym"], rec["err"])
    return (matches, domains, n_ranges, range_size, framerate, sampwidth, tile_size, domain_step, energy_threshold,
            original_len)
