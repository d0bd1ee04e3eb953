"""Time the similarity search kernel with diagnostic ablations (tools only; outputs are wrong for dbg & 7 != 0).

dbg bits (k_sim_topk_f16, STATS build): 1 = no slow path, 2 = skip MFMA + filter, 4 = no chunk DMA beyond one
chunk, 128 = DMA every other chunk, 256 = no group barrier, 512 = fold without ballots, 1024 = MFMA without fold.
usage: python tools/topk_ablate.py [seconds] [dbg,dbg,...] (geometry variants: tools/ab_build.sh + tools/ab_topk.py).
Counters: replayed chunks, firing tiles, appends, compactions, per-segment tick shares, overflow fallbacks."""
import os as _os_dbg
_os_dbg.environ.setdefault("FWAV_DEBUG_LIBRARY", "1")  # the search knobs: libfwav_debug.so
import os, sys, time
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "audio-compression_amd")]
import torch
import __graft_entry__
__graft_entry__.build()
from fwav import engine, synth
from fwav._lib import call

secs = float(sys.argv[1]) if len(sys.argv) > 1 else 60.0
sig = torch.from_numpy(synth.noise(secs, 44100)).cuda()
r = engine.compress_device(sig, 2048, 64, keep_intermediates=True)
torch.cuda.synchronize()
nd, nr = r.n_domains, r.n_ranges
emb16 = torch.empty(2 * ((nd + 255) // 256) * 256 * 16, dtype=torch.float16, device="cuda")
# rebuild emb16 through the pool+embed entry point
r2 = engine.compress_device(sig, 2048, 64, keep_intermediates=True)
st = torch.cuda.current_stream().cuda_stream
tab = engine.embed_tables(8, torch.device("cuda"))
pool = torch.empty(nd * 8, device="cuda"); emb = torch.empty(nd * 16, device="cuda")
ws = torch.empty(16 << 20, dtype=torch.uint8, device="cuda")
call("fwav_pool_embed", sig.data_ptr(), sig.numel(), 2048, 8, 2, tab.data_ptr(), pool.data_ptr(), emb.data_ptr(),
     emb16.data_ptr(), ws.data_ptr(), ws.numel(), st)
active = torch.arange(nr, dtype=torch.int32, device="cuda")
n_active = torch.tensor([nr], dtype=torch.int32, device="cuda")
cand = torch.empty(nr * 64, dtype=torch.int32, device="cuda")
from fwav._lib import size_call
wsk = torch.empty(size_call("fwav_sim_topk_workspace_size", nr, nd, 64), dtype=torch.uint8, device="cuda")
stats = torch.zeros(16, dtype=torch.int64, device="cuda")  # kStats = 12 used
call("fwav_debug_sim_topk", emb.data_ptr(), emb16.data_ptr(), nd, active.data_ptr(), n_active.data_ptr(), nr, 0,
     64, cand.data_ptr(), wsk.data_ptr(), wsk.numel(), 0, stats.data_ptr(), st)
torch.cuda.synchronize()
sv = stats.cpu().tolist()
waves = (nr + 255) // 256 * 8
us = lambda t: t / 100.0 / waves  # noqa: E731  (100 MHz ticks → µs per wave)
print("per wave: slow_chunk calls %.1f, firing tiles %.1f, appends/query %.1f, compactions/query %.2f" %
      (sv[0] / waves, sv[1] / waves, sv[2] / nr, sv[3] / nr))
tot = sv[6]
print("per-wave share of kernel ticks: barrier %.3f, streaming %.3f, replays %.3f (of which compactions %.3f, "
      "appends %.3f, fragment loads %.3f), final %.3f, other %.3f" %
      (sv[7] / tot, sv[9] / tot, sv[4] / tot, sv[5] / tot, sv[10] / tot, sv[11] / tot, sv[8] / tot,
       1 - (sv[7] + sv[9] + sv[4] + sv[8]) / tot), flush=True)
for dbg in (1, 4):
    stats.zero_()
    call("fwav_debug_sim_topk", emb.data_ptr(), emb16.data_ptr(), nd, active.data_ptr(), n_active.data_ptr(), nr, 0,
         64, cand.data_ptr(), wsk.data_ptr(), wsk.numel(), dbg, stats.data_ptr(), st)
    torch.cuda.synchronize()
    sv = stats.cpu().tolist()
    tot = sv[6]
    o = wsk.numel() - 4 - 4 * nr  # workspace tail: ovf list, its count, then u32 seeds[q]
    n_ovf = int(wsk[o:o + 4].view(torch.int32).item())
    print("dbg=%d: overflowed queries (exact-mode relaunch) %d" % (dbg, n_ovf))
    print("dbg=%d: replays/wave %.0f firing tiles/wave %.0f appends/q %.0f compactions/q %.2f | shares: barrier %.3f, "
          "streaming %.3f, replays %.3f, final %.3f, other %.3f" %
          (dbg, sv[0] / waves, sv[1] / waves, sv[2] / nr, sv[3] / nr, sv[7] / tot, sv[9] / tot, sv[4] / tot,
           sv[8] / tot, 1 - (sv[7] + sv[9] + sv[4] + sv[8]) / tot), flush=True)
for dbg in ([int(x) for x in sys.argv[2].split(',')] if len(sys.argv) > 2 else [0, 1, 4, 5, 128, 2, 0]):
    for rep in range(2):
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        call("fwav_debug_sim_topk", emb.data_ptr(), emb16.data_ptr(), nd, active.data_ptr(), n_active.data_ptr(), nr, 0,
             64, cand.data_ptr(), wsk.data_ptr(), wsk.numel(), dbg, None, st)
        e1.record(); torch.cuda.synchronize()
    print(f"dbg={dbg}: {e0.elapsed_time(e1):.2f} ms", flush=True)
