"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself (this container only).

Run:  python tests/golden/make_golden.py            (needs /root/reference; never runs on the GPU box)

How the reference is driven: ``fractal.py`` is imported from /root/reference with
an inert ``librosa`` module whose ``filters.mel`` returns zeros.  librosa is absent from the image; its
only consumer is ``get_mel_filterbank`` (fractal.py:522-525), whose output is handed to ``gpu_worker``
(fractal.py:1210-1232) and never read (fractal.py:637-754), so it cannot influence any value recorded
here.  The pipeline is then called stage by stage in-process — the reference's own functions, in the
order ``compress_audio`` calls them (fractal.py:1070-1245) — which the survey measured bit-exact against
the forked ``compress_audio``; the tone case below re-checks that against a real ``compress_audio`` call.

Each ``<case>.npz`` holds only data (inputs and reference outputs):
  params      json: framerate, sampwidth, tile, rs, step, thr, K list, n_ranges, n_domains
  signal      f32[N]        input
  voiced      u8[N]         voiced_detection mask (fractal.py:880-909)
  ranges      f32[nr, rs]   voiced-masked, reflect-padded ranges (fractal.py:1079-1112)
  pool        f32[nd, rs]   build_domains_memmap (fractal.py:285-334)
  emb         f32[nd, 16]   build_domain_embeddings (fractal.py:238-280)
  for each K:  cand_K i32[nr,K] (cpu_worker, fractal.py:556-632), kth_K/k1th_K f32[nr] (K-th and (K+1)-th
               reference score, for the near-tie rule of SURVEY Appendix A), m_idx_K/m_s_K/m_o_K/m_sym_K/
               m_err_K (the (domain, s, o, sym, err) tuples of _process_gpu_batch, fractal.py:757-850),
               dec_K f32 + dec_iters_K (decompress_audio defaults, fractal.py:1378-1473),
               dec50_K f32 (iterations=50, eps=0), decd_K f32 + decd_iters_K (s_damping=0.3, eps=0, 12 iters)
  fwav_K      u8[...]       save_compressed bytes (fractal.py:1278-1322), small cases only
"""
from __future__ import annotations

import json
import logging
import os
import sys
import tempfile
import time
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "audio-compression_amd"))
from fwav import synth  # noqa: E402


def _import_reference():
    lib = types.ModuleType("librosa")
    filt = types.ModuleType("librosa.filters")
    filt.mel = lambda sr=None, n_fft=2048, n_mels=128, fmin=0.0, fmax=None, **kw: np.zeros(
        (n_mels, 1 + n_fft // 2), np.float32)
    lib.filters = filt
    sys.modules["librosa"] = lib
    sys.modules["librosa.filters"] = filt
    sys.path.insert(0, "/root/reference")
    import fractal as F  # noqa: E402
    return F


class ListQueue:
    def __init__(self):
        self.items = []

    def put(self, x):
        self.items.append(x)


class IterCapture(logging.Handler):
    def __init__(self):
        super().__init__(level=logging.DEBUG)
        self.msgs = []

    def emit(self, record):
        self.msgs.append(record.getMessage())


def run_decode(F, matches, pool, nr, rs, orig_len, **kw):
    h = IterCapture()
    lg = logging.getLogger("fwavc")
    old = lg.level
    lg.setLevel(logging.DEBUG)
    lg.addHandler(h)
    try:
        out = np.asarray(F.decompress_audio(matches, pool, nr, rs, original_len=orig_len, **kw), np.float32)
    finally:
        lg.removeHandler(h)
        lg.setLevel(old)
    iters = sum(1 for m in h.msgs if m.startswith("Iteration "))
    deltas = [float(m.split("delta=")[1]) for m in h.msgs if m.startswith("Iteration ")]
    return out, iters, np.array(deltas, np.float64)


def staged(F, signal, tile, thr, Ks, with_fwav, framerate, sampwidth):
    rs = max(4, tile // 256)
    step = max(1, rs // 4)
    vm = F.voiced_detection(signal, frame_size=rs * 2, energy_threshold=thr)
    ws = signal * vm
    orig = len(ws)
    pad = (rs - orig % rs) % rs
    if pad:
        ws = np.pad(ws, (0, pad), mode="reflect")
    nr = len(ws) // rs
    ranges = ws.reshape(nr, rs)
    tmp = tempfile.mkdtemp()
    dpath, nd = F.build_domains_memmap(signal, tile, rs, step, block_size=500, tmpdir=tmp)
    epath = F.build_domain_embeddings(dpath, nd, rs, emb_dim=16, block_size=4096, tmpdir=tmp)
    pool = np.array(np.memmap(dpath, dtype="float32", mode="r", shape=(nd, rs)))
    emb = np.array(np.memmap(epath, dtype="float32", mode="r", shape=(nd, 16)))
    out = dict(signal=signal, voiced=vm.astype(np.uint8), ranges=np.ascontiguousarray(ranges), pool=pool,
               emb=emb)
    pool_mm = np.memmap(dpath, dtype="float32", mode="r", shape=(nd, rs))
    for K in Ks:
        F.top_k = K
        q = ListQueue()
        F.cpu_worker(idx_slice=np.arange(nr), ranges=ranges,
                     range_embs=np.memmap(epath, dtype="float32", mode="r", shape=(nr, 16)),
                     domain_embs_path=epath, n_domains=nd, emb_dim=16, candidate_queue=q,
                     ann_index_path=None, energy_thresh=thr, fast_mode=True, batch_size=128)
        pairs = [p for b in q.items if b is not None for p in b]
        assert len(pairs) == nr
        cand = np.stack([c for _, c in sorted(pairs, key=lambda t: t[0])]).astype(np.int32)
        # reference scores for the near-tie rule (same sgemv call as fractal.py:537)
        dom_embs = np.memmap(epath, dtype="float32", mode="r", shape=(nd, 16))
        kth = np.full(nr, np.nan, np.float32)
        k1th = np.full(nr, np.nan, np.float32)
        for i in range(nr):
            if cand[i, 0] < 0:
                continue
            sc = np.sort(dom_embs @ emb[i])[::-1]
            kth[i] = sc[min(K, nd) - 1]
            if nd > K:
                k1th[i] = sc[K]
        rq = ListQueue()
        for s in range(0, nr, 512):
            F._flush_gpu_batch(pairs[s:s + 512], ranges, pool_mm, rq, use_gpu=False)
        res = dict(rq.items)
        matches = [res[i] for i in range(nr)]
        out[f"cand_{K}"] = cand
        out[f"kth_{K}"] = kth
        out[f"k1th_{K}"] = k1th
        out[f"m_idx_{K}"] = np.array([m[0] for m in matches], np.int32)
        out[f"m_s_{K}"] = np.array([m[1] for m in matches], np.float32)
        out[f"m_o_{K}"] = np.array([m[2] for m in matches], np.float32)
        out[f"m_sym_{K}"] = np.array([m[3] for m in matches], np.uint8)
        out[f"m_err_{K}"] = np.array([m[4] for m in matches], np.float32)
        d, it, dl = run_decode(F, matches, pool, nr, rs, orig)
        out[f"dec_{K}"], out[f"dec_iters_{K}"], out[f"dec_deltas_{K}"] = d, np.int32(it), dl
        d, it, dl = run_decode(F, matches, pool, nr, rs, orig, iterations=50, convergence_eps=0.0)
        out[f"dec50_{K}"], out[f"dec50_deltas_{K}"] = d, dl
        d, it, dl = run_decode(F, matches, pool, nr, rs, orig, iterations=12, convergence_eps=0.0,
                               s_damping=0.3)
        out[f"decd_{K}"], out[f"decd_iters_{K}"], out[f"decd_deltas_{K}"] = d, np.int32(it), dl
        if with_fwav:
            fp = os.path.join(tmp, "x.fwav")
            F.save_compressed(fp, matches, pool, rs, framerate, sampwidth, tile, step, thr, orig)
            out[f"fwav_{K}"] = np.frombuffer(open(fp, "rb").read(), np.uint8)
    for p in (dpath, epath):
        os.remove(p)
    params = dict(framerate=framerate, sampwidth=sampwidth, tile=tile, rs=rs, step=step, thr=thr, Ks=list(Ks),
                  n_ranges=int(nr), n_domains=int(nd), original_len=int(orig))
    out["params"] = np.array(json.dumps(params))
    return out


def main():
    F = _import_reference()
    cases = {
        # name: (signal, framerate, sampwidth, tile, thr, Ks, with_fwav)
        "tone": (synth.tone(), 8000, 2, 128, 1e-4, (32,), True),
        "sweep": (synth.sweep(1.0, 16000), 16000, 2, 512, 1e-4, (32, 64), True),
        "noise2048": (synth.noise(1.0, 44100), 44100, 4, 2048, 1e-4, (64,), False),
        "noise4096": (synth.noise(1.0, 44100), 44100, 4, 4096, 1e-4, (64,), False),
        "speech4096": (synth.speech_like(2.0, 44100, seed=1, floor=False), 44100, 4, 4096, 1e-4, (64,), False),
        # ragged length (reflect pad of the last range) and an odd tile, K larger than the pool
        "ragged": (synth.noise(0.05, 44100, seed=3)[:2203], 44100, 4, 1000, 1e-4, (16, 2000), True),
        # fewer than 5 voiced-detection frames (30 samples, frame 8): np.convolve swaps its operands
        "tiny": (synth.noise(30 / 8000, 8000, seed=9), 8000, 4, 16, 1e-4, (8,), True),
    }
    only = sys.argv[1:]
    for name, (sig, fr, sw, tile, thr, Ks, wf) in cases.items():
        if only and name not in only:
            continue
        t0 = time.time()
        out = staged(F, sig, tile, thr, Ks, wf, fr, sw)
        np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **out)
        print(name, json.loads(str(out["params"])), f"{time.time() - t0:.1f}s", flush=True)

    # cross-check: the staged harness equals the forked compress_audio (tone, K = 32 module default)
    if not only or "tone" in only:
        F.top_k = 32
        sig = synth.tone()
        res = F.compress_audio(sig, 8000, 2, tile_size=128, energy_thresh=1e-4, use_gpu=False)
        g = np.load(os.path.join(HERE, "tone.npz"))
        m = res[0]
        assert np.array_equal(np.array([x[0] for x in m], np.int32), g["m_idx_32"])
        assert np.array_equal(np.array([x[2] for x in m], np.float32).view(np.uint32), g["m_o_32"].view(np.uint32))
        print("staged harness == forked compress_audio on tone: OK")

    # edge cases of the API surface (fractal.py:1083-1093, 1130-1140, and the nr > nd mmap error)
    edges = {}
    F.top_k = 32
    short = synth.noise(0.01, 44100, seed=5)  # N=441 < tile → empty tuple
    r = F.compress_audio(short, 44100, 4, tile_size=2048, use_gpu=False)
    edges["short"] = dict(n_matches=len(r[0]), pool_shape=list(r[1].shape), rest=[int(r[2]), int(r[3]), int(r[4]),
                                                                                    int(r[5]), float(r[6]), int(r[7])])
    silent = np.zeros(5000, np.float32)
    r = F.compress_audio(silent, 44100, 4, tile_size=1024, use_gpu=False)
    edges["silent"] = dict(n_matches=len(r[0]), pool_shape=list(r[1].shape), rest=[int(r[2]), int(r[3]), int(r[4]),
                                                                                     int(r[5]), float(r[6]), int(r[7])])
    try:
        F.compress_audio(synth.noise(1.0, 44100)[:2448], 44100, 4, tile_size=2048, use_gpu=False)
        edges["q9"] = dict(raised=None)
    except Exception as e:  # noqa: BLE001
        edges["q9"] = dict(raised=type(e).__name__, msg=str(e))
    with open(os.path.join(HERE, "edges.json"), "w") as f:
        json.dump(edges, f, indent=1)
    print("edges", edges)


if __name__ == "__main__":
    main()
