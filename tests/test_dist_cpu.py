"""World-size-2/3 gloo tests of the range-sharded compress and decompress (fwav.dist) on CPU.

The per-rank compute is the oracle restatement (tests may use the oracle as the checker/compute stand-in;
the product path plugs in the HIP engine).  The communication code — signal broadcast, prune-balanced blocks,
SoA gather; pool broadcast, match scatter, per-chunk all-reduce of Δ partials, reconstruction gather — is the
product code, and its output must equal a single-process oracle run.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _oracle_compute(sig, tile_size, top_k, energy_thresh, shard):
    from oracle import fractal_oracle as O
    r = O.compress(sig.cpu().numpy(), tile_size, top_k, energy_thresh)
    rs = r["rs"]
    nr = len(r["idx"])
    lo, hi = shard(torch.from_numpy(np.ascontiguousarray(r["ranges"].reshape(-1))), nr, rs)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a[lo:hi]))  # noqa: E731
    return dict(idx=t(r["idx"]), s=t(r["s"]), o=t(r["o"]), sym=t(r["sym"]), err=t(r["err"]),
                pool=torch.from_numpy(r["pool"]), silent=lambda: False)


def _worker(rank, world, port, sig, tile, k, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "audio-compression_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from fwav.dist import compress_sharded
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = compress_sharded(sig if rank == 0 else None, tile, k, 1e-4, device=torch.device("cpu"),
                           compute=_oracle_compute)
    if rank == 0:
        q.put({kk: v for kk, v in out.items() if kk != "pool"})
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_equals_single_process(world):
    from fwav import synth
    from oracle import fractal_oracle as O
    sig = synth.speech_like(1.5, 16000, seed=2, floor=False)
    tile, k = 1024, 16
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, sig, tile, k, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = None
    import queue as _q
    for _ in range(240):
        try:
            out = q.get(timeout=1)
            break
        except _q.Empty:
            if any(p.exitcode not in (None, 0) for p in procs):
                break
    for p in procs:
        p.join(timeout=60)
        if p.exitcode is None:
            p.kill()
    assert out is not None, "a rank failed"
    assert all(p.exitcode == 0 for p in procs)
    ref = O.compress(sig, tile, k)
    for f in ("idx", "s", "o", "sym", "err"):
        a, b = np.asarray(out[f]), np.asarray(ref[f])
        assert a.shape == b.shape
        assert np.array_equal(a.view(np.uint8), b.view(np.uint8)), f
    blocks = out["blocks"]
    assert blocks[0][0] == 0 and blocks[-1][1] == len(ref["idx"])
    assert all(blocks[i][1] == blocks[i + 1][0] for i in range(world - 1))


def _pipelined_worker(rank, world, port, sigs, tile, k, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "audio-compression_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from fwav.dist import compress_sharded_finish, compress_sharded_start
    dist.init_process_group("gloo", rank=rank, world_size=world)
    waited = []

    def compute(sig, tile_size, top_k, thr, shard):
        r = _oracle_compute(sig, tile_size, top_k, thr, shard)
        tag = len(waited)
        waited.append(False)
        # a deferred result: err is only final once wait() ran (as with engine.compress_device(defer_ties=True))
        final = r["err"].clone()
        r["err"] = torch.full_like(final, float("nan"))

        def wait():
            r["err"].copy_(final)
            waited[tag] = True
        r["wait"] = wait
        return r

    outs, inflight = [], []
    for sg in sigs:  # two calls in flight, finished in order (bench.py's multi-rank timed loop)
        inflight.append(compress_sharded_start(torch.from_numpy(sg) if rank == 0 else None, tile, k, 1e-4,
                                               device=torch.device("cpu"), compute=compute, n=len(sg)))
        while len(inflight) > 2:
            outs.append(compress_sharded_finish(inflight.pop(0)))
    outs += [compress_sharded_finish(h) for h in inflight]
    if rank == 0:
        q.put(dict(outs=[{kk: np.asarray(v) for kk, v in o.items() if kk in ("idx", "s", "o", "sym", "err")}
                         for o in outs], waited=waited))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_pipelined_start_finish_equals_single_process():
    """compress_sharded_start/finish with two calls in flight: each call's gathered arrays equal a single-process
    run on its own signal, and each deferred result was completed before its gather."""
    from fwav import synth
    from oracle import fractal_oracle as O
    sigs = [synth.speech_like(0.6, 16000, seed=s, floor=False) for s in (3, 4, 5, 6)]
    tile, k, world = 1024, 8, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipelined_worker, args=(r, world, port, sigs, tile, k, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = None
    import queue as _q
    for _ in range(240):
        try:
            out = q.get(timeout=1)
            break
        except _q.Empty:
            if any(p.exitcode not in (None, 0) for p in procs):
                break
    for p in procs:
        p.join(timeout=60)
        if p.exitcode is None:
            p.kill()
    assert out is not None, "a rank failed"
    assert all(p.exitcode == 0 for p in procs)
    assert out["waited"] == [True] * len(sigs)
    assert len(out["outs"]) == len(sigs)
    for sg, got in zip(sigs, out["outs"]):
        ref = O.compress(sg, tile, k)
        for f in ("idx", "s", "o", "sym", "err"):
            assert np.array_equal(got[f].view(np.uint8), np.asarray(ref[f]).view(np.uint8)), f


def test_balanced_bounds():
    from fwav.dist import balanced_bounds
    w = np.r_[np.zeros(1000), np.ones(1000), np.zeros(500), np.ones(1000)]
    b = balanced_bounds(w, 4)
    assert b[0][0] == 0 and b[-1][1] == len(w)
    loads = [w[a:c].sum() for a, c in b]
    assert max(loads) - min(loads) <= 2
    assert balanced_bounds(np.zeros(10), 3)[-1][1] == 10


def test_prune_balanced_bounds():
    from fwav.dist import prune_balanced_bounds
    rs = 4
    x = np.zeros((4000, rs), np.float32)
    x[1000:2000] = 0.1       # active (mean r² = 1e-2 >= 7.5e-5)
    x[3000:4000] = 0.1
    b = prune_balanced_bounds(torch.from_numpy(x.reshape(-1)), 4000, rs, 1e-4, 2)
    assert b[0][0] == 0 and b[-1][1] == 4000 and b[0][1] == b[1][0]
    assert 1900 <= b[0][1] <= 3100  # half of the active ranges on each side
    act = (x.astype(np.float64) ** 2).mean(1) >= np.float32(0.75e-4)
    loads = [act[a:c].sum() for a, c in b]
    assert abs(loads[0] - loads[1]) <= 2


# ------------------------------------------------------------------------------------------------- decompress
SPAN = 512  # small canonical block so the test signals span several blocks per rank


class CpuChunkDecoder:
    """numpy stand-in for fwav.dist.ShardDecoder (test infrastructure): decompress_audio arithmetic in numpy order
    (fractal.py:1411-1467, as oracle.decode) over chunks of 64 iterations, per-block Δ partials laid out like
    fwav_decode_run's, a fixed-order block sum, and the stopping chunk recomputed from its start state."""

    CI = 64

    def __init__(self, idx, s, o, sym, pool, lo, nr, rs, iterations, eps, s_clip=16.0, s_damping=0.0, init=None):
        from oracle import fractal_oracle as O
        self.args = (idx, s, o, sym, pool, lo, nr, rs)
        self.O = O
        F32 = np.float32
        idx = idx.numpy().copy()
        s = s.numpy().astype(F32).copy()
        o = o.numpy().astype(F32).copy()
        sym = sym.numpy().astype(bool).copy()
        pool = pool.numpy().reshape(-1, rs)
        inval = idx < 0
        idx[inval] = 0
        tiles = pool[idx] if len(idx) else np.zeros((0, rs), F32)
        tiles[inval] = 0
        s[inval] = 0
        o[inval] = 0
        sym[inval] = False
        self.T = np.where(sym[:, None], tiles[:, ::-1], tiles)
        self.tc = self.T - O.pw_mean(self.T)[:, None]
        self.den = O.pw_sum(self.tc * self.tc)
        self.valid = self.den > F32(1e-12)
        self.s, self.o = s, o
        self.m, self.lo, self.nr, self.rs = len(idx), lo, nr, rs
        self.iterations, self.eps = iterations, eps
        self.c, self.damp = abs(F32(s_clip)), s_damping
        self.first = 2 if (eps > 0 and iterations > 2) else self.CI  # fwav_decode.hip dec_first
        self.n_chunks = 0 if iterations <= 0 else (1 if iterations <= self.first else
                                                   1 + -(-(iterations - self.first) // self.CI))
        self.nblk = -(-max(nr, 1) // SPAN)
        self.part = torch.zeros(self.CI * self.nblk * 2, dtype=torch.float64)
        self.rec = np.zeros((self.m, rs), F32) if init is None else init.numpy().reshape(self.m, rs).copy()
        self.start = self.rec
        self.deltas, self.ran, self.stopped, self.prev = [], 0, False, None

    def _t0(self, c):
        return 0 if c == 0 else self.first + (c - 1) * self.CI

    def _len(self, c):
        return min(self.first if c == 0 else self.CI, self.iterations - self._t0(c))

    def _step(self, rec):
        F32 = np.float32
        rc = rec - self.O.pw_mean(rec)[:, None]
        num = self.O.pw_sum(rc * self.tc)
        s_opt = np.zeros(self.m, F32)
        s_opt[self.valid] = num[self.valid] / self.den[self.valid]
        su = F32(1.0 - self.damp) * self.s + F32(self.damp) * s_opt if self.damp > 0 else \
            np.where(self.valid, s_opt, self.s)
        su = np.clip(su, -self.c, self.c)
        return F32(0.0) + (su[:, None] * self.T + self.o[:, None])

    def run(self, chunk):
        if self.stopped:
            return
        self.part.zero_()
        self.start = self.rec
        p = self.part.view(self.CI, self.nblk, 2).numpy()
        blk = (self.lo + np.arange(self.m)) // SPAN
        rec = self.rec
        for t in range(self._len(chunk)):
            nxt = self._step(rec)
            np.add.at(p[t, :, 0], blk, (rec.astype(np.float64) ** 2).sum(1))  # sequential, in range order
            np.add.at(p[t, :, 1], blk, ((nxt - rec).astype(np.float64) ** 2).sum(1))
            rec = nxt
        self.rec = rec

    def partials_prefix(self):
        return self.part

    def reduce(self, chunk):
        if self.stopped:
            return
        from fwav.dist import decode_beta, decode_decision
        p = self.part.view(self.CI, self.nblk, 2).numpy()
        for t in range(self._len(chunk)):
            rn, dn = float(np.sum(p[t, :, 0])), float(np.sum(p[t, :, 1]))
            d = np.sqrt(dn) / (np.sqrt(rn) if rn > 0 else 1.0)
            self.deltas.append(d)
            self.ran = self._t0(chunk) + t + 1
            dec = decode_decision(rn, dn, d, self.eps, decode_beta(self.nr * self.rs))
            if dec != 0:
                self.stopped = True
                rec = self.start
                for _ in range(t):
                    rec = self._step(rec)
                self.prev = rec if dec == 2 else None
                self.rec = self._step(rec)
                return

    def finish(self):
        pend = None if self.prev is None else torch.from_numpy(self.prev.reshape(-1).copy())
        return torch.from_numpy(self.rec.reshape(-1).copy()), self.ran, self.deltas, pend

    def exact_delta(self, prev, nxt):
        d = self.O.reference_delta(prev.numpy(), nxt.numpy())
        return d, d < self.eps

    def resumed(self, rec, left):
        return CpuChunkDecoder(*self.args, left, self.eps, float(self.c), self.damp, init=rec)


def _dec_worker(rank, world, port, soa, pool, nr, rs, kw, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "audio-compression_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from fwav.dist import decompress_sharded
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = decompress_sharded(soa if rank == 0 else None, pool if rank == 0 else None, nr, rs,
                             device=torch.device("cpu"), decoder=CpuChunkDecoder, span=SPAN, **kw)
    if rank == 0:
        q.put((out[0], out[1]))
    dist.barrier()
    dist.destroy_process_group()


def _run_world(target, world, args):
    import queue as _q
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, *args, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = None
    for _ in range(240):
        try:
            out = q.get(timeout=1)
            break
        except _q.Empty:
            if any(p.exitcode not in (None, 0) for p in procs):
                break
    for p in procs:
        p.join(timeout=60)
        if p.exitcode is None:
            p.kill()
    assert out is not None, "a rank failed"
    assert all(p.exitcode == 0 for p in procs)
    return out


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_decompress_equals_oracle(world):
    """Pool broadcast, match scatter, per-chunk Δ all-reduce, reconstruction gather: the gathered reconstruction
    equals the oracle's decode bit-for-bit with the same iteration count, for a stop at 2 (defaults), a stop inside
    the second chunk and a forced run; Δ equals the single-process chunk decoder exactly (one canonical sum order)."""
    from oracle import fractal_oracle as O
    rng = np.random.default_rng(world)
    nr, nd, rs = 3000, 700, 8
    pool = rng.normal(0, 0.3, (nd, rs)).astype(np.float32)
    soa = dict(idx=rng.integers(0, nd, nr).astype(np.int32), s=rng.uniform(-1, 1, nr).astype(np.float32),
               o=rng.normal(0, 0.1, nr).astype(np.float32), sym=(rng.random(nr) < 0.5).astype(np.uint8))
    soa["idx"][::41] = -1
    for kw in (dict(), dict(iterations=300, convergence_eps=1e-6, s_damping=0.9),
               dict(iterations=70, convergence_eps=0.0, s_damping=0.3)):
        rec, info = _run_world(_dec_worker, world, (soa, pool, nr, rs, kw))
        ref, it, rdel = O.decode(soa["idx"], soa["s"], soa["o"], soa["sym"], pool, nr, rs, **kw)
        assert info["iterations"] == it
        assert np.array_equal(rec.view(np.uint32), ref.view(np.uint32))
        # f64 Δ, except at an iteration the exact check decided (the reference's float32 value there)
        np.testing.assert_allclose(info["deltas"], rdel, rtol=1e-6)


def test_decode_bounds_aligned():
    from fwav.dist import decode_bounds
    for nr, world in ((21_600_000, 8), (330_750, 3), (5000, 4), (0, 2), (4096, 3)):
        b = decode_bounds(nr, world, 4096)
        assert b[0][0] == 0 and b[-1][1] == nr
        assert all(b[i][1] == b[i + 1][0] for i in range(world - 1))
        assert all(a % 4096 == 0 for a, _ in b)
        sizes = [c - a for a, c in b]
        assert max(sizes) - min(sizes) <= 4096 or nr < 4096 * world


@pytest.mark.parametrize("side", ["stop", "go_on"])
def test_sharded_decompress_exact_check(side):
    """The early exit where the f64 Δ cannot decide (fractal.py:1460-1465): eps placed inside the certified band of an
    iteration whose reference Δ (float32 BLAS sdot norms) and f64 Δ differ — just above the reference's Δ (it stops
    there) or just below it (it goes on: every rank resumes from its slice).  Two gloo ranks take the reference's
    decision (the oracle's iteration count and reconstruction, bit for bit)."""
    from fwav.dist import decode_beta
    from oracle import fractal_oracle as O
    rng = np.random.default_rng(11)
    nr, nd, rs = 3000, 700, 8
    pool = rng.normal(0, 0.3, (nd, rs)).astype(np.float32)
    soa = dict(idx=rng.integers(0, nd, nr).astype(np.int32), s=rng.uniform(-1, 1, nr).astype(np.float32),
               o=rng.normal(0, 0.1, nr).astype(np.float32), sym=(rng.random(nr) < 0.5).astype(np.uint8))
    base = dict(iterations=40, s_damping=0.5)
    args = (soa["idx"], soa["s"], soa["o"], soa["sym"], pool, nr, rs)
    _, _, d64 = O.decode(*args, convergence_eps=0.0, **base)
    _, _, dref = O.decode(*args, convergence_eps=0.0, deltas="reference", **base)
    beta = decode_beta(nr * rs)
    t = next(t for t in range(5, 40) if dref[t] != d64[t])
    eps = dref[t] * (1 + beta / 4) if side == "stop" else dref[t] * (1 - beta / 4)
    assert abs(eps - d64[t]) < beta * d64[t]  # inside the band: the device cannot decide on its own
    kw = dict(base, convergence_eps=eps)
    ref, it, _ = O.decode(*args, **kw)
    assert (it == t + 1) == (side == "stop")
    rec, info = _run_world(_dec_worker, 2, (soa, pool, nr, rs, kw))
    assert info["iterations"] == it
    assert np.array_equal(rec.view(np.uint32), ref.view(np.uint32))
    assert info["deltas"][t] == dref[t]  # the checked iteration reports the reference's own Δ
