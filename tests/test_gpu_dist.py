"""Multi-rank rehearsal of fwav.dist on ONE GPU: two gloo ranks share cuda:0 and run the product HIP compute
(compress_device on a prune-balanced shard; ShardDecoder with the per-chunk all-reduce of Δ partials).  The
gathered results must equal the single-GPU compress / decode bit-for-bit — the same check the driver's 8-GPU RCCL
runs rely on (there, only the collective backend differs)."""
import os
import socket
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ("idx", "s", "o", "sym", "err")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, cfg, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "audio-compression_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from fwav import dist as D, engine, synth
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        sig = synth.make_config_signal(cfg["config"], seconds=cfg["seconds"], seed=3)[0]
        tile, K = cfg["tile"], cfg["K"]
        out = D.compress_sharded(sig if rank == 0 else None, tile, K, 1e-4, device=dev)
        dec = D.decompress_sharded(out if rank == 0 else None, out["pool"] if rank == 0 else None,
                                   out["n_ranges"] if rank == 0 else 0, out["range_size"] if rank == 0 else 0,
                                   iterations=150, convergence_eps=1e-6, s_damping=0.9, original_len=len(sig),
                                   device=dev)
        if rank == 0:
            one = engine.compress_device(torch.from_numpy(sig).to(dev), tile, K)
            same = {f: bool(np.array_equal(out[f].view(np.uint8), getattr(one, f).cpu().numpy().view(np.uint8)))
                    for f in FIELDS}
            rec1, ran1, del1 = engine.decompress_device(one.idx, one.s, one.o, one.sym, one.pool, one.n_ranges,
                                                        one.range_size, 150, 1e-6, s_damping=0.9)
            rec, info = dec
            q.put(dict(same=same, blocks=out["blocks"], dec_same=bool(np.array_equal(
                rec.view(np.uint32), rec1.cpu().numpy()[:len(sig)].view(np.uint32))),
                ran=(info["iterations"], ran1), deltas_same=info["deltas"] == del1, dblocks=info["blocks"]))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put(dict(error=repr(e)))
        raise


@pytest.mark.parametrize("cfg", [dict(config="cfg2", seconds=2.0, tile=2048, K=64),
                                 dict(config="cfg3", seconds=3.0, tile=4096, K=64)])
def test_two_ranks_share_gpu(cfg):
    import queue as _q
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, cfg, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = None
    for _ in range(170):
        try:
            out = q.get(timeout=1)
            break
        except _q.Empty:
            if any(p.exitcode not in (None, 0) for p in procs):
                break
    for p in procs:
        p.join(timeout=30)
        if p.exitcode is None:
            p.kill()
    assert out is not None and "error" not in out, out
    assert all(out["same"].values()), out["same"]
    (a0, b0), (a1, b1) = out["blocks"]
    assert a0 == 0 and b0 == a1 and b0 > 0
    assert out["dec_same"] and out["ran"][0] == out["ran"][1] and out["deltas_same"]
    assert out["dblocks"][0][1] % 4096 == 0


def _long_range_worker(rank, world, port, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "audio-compression_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from fwav import dist as D, engine, synth
    try:
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        sig = synth.noise(1.0, 44100, seed=9)
        one = engine.compress_device(torch.from_numpy(sig).to(dev), 16384, 16)  # rs = 64 > 32
        m = {f: getattr(one, f).cpu().numpy() for f in ("idx", "s", "o", "sym")} if rank == 0 else None
        dom = one.pool.view(-1, one.range_size).cpu().numpy() if rank == 0 else None
        out = D.decompress_sharded(m, dom, one.n_ranges if rank == 0 else 0, one.range_size if rank == 0 else 0,
                                   iterations=8, convergence_eps=1e-3, device=dev)
        if rank == 0:
            rec1, ran1, del1 = engine.decompress_device(one.idx, one.s, one.o, one.sym, one.pool, one.n_ranges,
                                                        one.range_size, 8, 1e-3)
            rec, info = out
            q.put(dict(same=bool(np.array_equal(rec.view(np.uint32), rec1.cpu().numpy().view(np.uint32))),
                       ran=(info["iterations"], ran1), rs=one.range_size))
        else:
            q.put(dict(rank1=out))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # noqa: BLE001
        q.put(dict(error=repr(e)))
        raise


def test_sharded_decode_long_ranges_falls_back_to_rank0():
    """range_size > 32 (tile ≥ 8448): the range-sharded kernels keep a range in registers and cannot take it, so every
    rank learns rs from the first broadcast and rank 0 decodes alone with the single-device streaming path — the
    result equals decompress_device, and no rank is left waiting in a collective."""
    import queue as _q
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_long_range_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    outs = []
    for _ in range(170):
        try:
            outs.append(q.get(timeout=1))
            if len(outs) == 2:
                break
        except _q.Empty:
            if any(p.exitcode not in (None, 0) for p in procs):
                break
    for p in procs:
        p.join(timeout=30)
        if p.exitcode is None:
            p.kill()
    assert len(outs) == 2 and not any("error" in o for o in outs), outs
    r0 = next(o for o in outs if "same" in o)
    assert r0["rs"] == 64 and r0["same"] and r0["ran"][0] == r0["ran"][1]
    assert next(o for o in outs if "rank1" in o)["rank1"] is None
