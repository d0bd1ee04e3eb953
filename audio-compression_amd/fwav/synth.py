"""Seeded synthetic inputs for the BASELINE.json configs (SURVEY.md §8(d) "Synthetic inputs").

The reference ships no audio, so every workload is generated here:

* cfg1  ``sweep``       1 s 16 kHz linear chirp 100→8000 Hz, int16-quantised (``sampwidth=2`` semantics,
                        integer units as ``read_wav_mono`` returns them, fractal.py:95-113).
* cfg2  ``noise``       60 s 44.1 kHz ``clip(N(0, 0.25²), −1, 1)``, ``default_rng(0)`` (float WAV semantics).
* cfg3  ``speech_like`` 10 min 44.1 kHz voiced syllables + fricatives + gaps (+ optional −60 dBFS floor).
* cfg4  ``noise``       60 min 48 kHz, same generator as cfg2.

A prefix of a longer ``noise`` signal equals the shorter one (numpy's generator is sequential), so golden
fixtures cut from 1 s slices describe the first second of the bench signal exactly.
"""
from __future__ import annotations

import numpy as np


def noise(seconds: float, sr: int = 44100, seed: int = 0, sigma: float = 0.25) -> np.ndarray:
    n = int(round(seconds * sr))
    rng = np.random.default_rng(seed)
    return np.clip(rng.normal(0.0, sigma, n), -1.0, 1.0).astype(np.float32)


def sweep(seconds: float = 1.0, sr: int = 16000, f0: float = 100.0, f1: float = 8000.0) -> np.ndarray:
    n = int(round(seconds * sr))
    t = np.arange(n, dtype=np.float64) / sr
    k = (f1 - f0) / (2.0 * seconds)
    x = np.round(0.5 * 32767.0 * np.sin(2.0 * np.pi * (f0 * t + k * t * t)))
    return x.astype(np.int16).astype(np.float32)


def tone(sr: int = 8000, dur: float = 0.12, freq: float = 440.0) -> np.ndarray:
    """The reference's own e2e fixture signal (test_e2e.py:6-10)."""
    t = np.linspace(0, dur, int(sr * dur), endpoint=False)
    amp = 0.5 * (2 ** 15 - 1)
    return (amp * np.sin(2 * np.pi * freq * t)).astype(np.int16).astype(np.float32)


def speech_like(seconds: float, sr: int = 44100, seed: int = 0, floor: bool = True) -> np.ndarray:
    """Speech-like signal: harmonic source on a wandering f0, syllable envelopes with gaps of digital
    silence, occasional fricative bursts; ``floor`` adds N(0, 1e-3) (−60 dBFS) so no pool row is exactly
    zero."""
    n = int(round(seconds * sr))
    rng = np.random.default_rng(seed)
    hop = int(0.05 * sr)
    n_knots = n // hop + 2
    steps = rng.normal(0.0, 8.0, n_knots)
    f0k = np.empty(n_knots)
    f0k[0] = 140.0
    for i in range(1, n_knots):
        f0k[i] = min(250.0, max(90.0, f0k[i - 1] + steps[i]))
    f0 = np.interp(np.arange(n, dtype=np.float64), np.arange(n_knots, dtype=np.float64) * hop, f0k)
    phase = 2.0 * np.pi * np.cumsum(f0) / sr
    src = np.zeros(n)
    for h in range(1, 13):
        src += np.sin(h * phase) / h
    env = np.zeros(n)
    fric = np.zeros(n)
    pos = 0
    while pos < n:
        dur = int(rng.uniform(0.12, 0.30) * sr)
        gap = int(rng.uniform(0.05, 0.25) * sr)
        seg = min(dur, n - pos)
        env[pos:pos + seg] = np.hanning(dur)[:seg]
        if rng.random() < 0.3:
            m = int(0.4 * dur)
            z = rng.normal(0.0, 1.0, m)
            fr = 0.3 * np.diff(z, prepend=0.0) * np.hanning(m)
            mm = min(m, seg)
            fric[pos:pos + mm] += fr[:mm]
        pos += dur + gap
    x = src * env
    x *= 0.5 / max(np.max(np.abs(x)), 1e-12)
    x += fric
    x *= 0.5 / max(np.max(np.abs(x)), 1e-12)
    if floor:
        x += rng.normal(0.0, 1e-3, n)
    return x.astype(np.float32)


#: BASELINE.json configs → (generator kwargs, framerate, sampwidth, tile_size, top_k)
CONFIGS = {
    "cfg1": dict(gen="sweep", seconds=1.0, sr=16000, sampwidth=2, tile=512, top_k=32),
    "cfg2": dict(gen="noise", seconds=60.0, sr=44100, sampwidth=4, tile=2048, top_k=64),
    "cfg3": dict(gen="speech_like", seconds=600.0, sr=44100, sampwidth=4, tile=4096, top_k=64),
    "cfg4": dict(gen="noise", seconds=3600.0, sr=48000, sampwidth=4, tile=2048, top_k=64),
}


def make_config_signal(name: str, seconds: float | None = None, seed: int = 0) -> tuple[np.ndarray, int, int]:
    c = CONFIGS[name]
    secs = c["seconds"] if seconds is None else seconds
    if c["gen"] == "sweep":
        return sweep(secs, c["sr"]), c["sr"], c["sampwidth"]
    if c["gen"] == "noise":
        return noise(secs, c["sr"], seed=seed), c["sr"], c["sampwidth"]
    return speech_like(secs, c["sr"], seed=seed), c["sr"], c["sampwidth"]
