"""Compare the fp16 search with the all-f32 kernel on a golden case under several work plans (tools only).
usage: python tools/diag_pieces.py [case] [K]"""
import os as _os_dbg
_os_dbg.environ.setdefault("FWAV_DEBUG_LIBRARY", "1")  # the search knobs: libfwav_debug.so
import os
import sys

sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "audio-compression_amd"),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests")]
import numpy as np
import torch

import __graft_entry__

__graft_entry__.build()
import fwav._lib as _L  # noqa: E402

if len(sys.argv) > 3:  # an A/B build (tools/ab_build.sh) in place of the in-tree library
    _L.LIB_PATH, _L._lib = os.path.abspath(sys.argv[3]), None
    print("library", _L.LIB_PATH)
from fwav import engine  # noqa: E402
from fwav._lib import call  # noqa: E402
from golden_util import load  # noqa: E402

case = sys.argv[1] if len(sys.argv) > 1 else "noise2048"
K = int(sys.argv[2]) if len(sys.argv) > 2 else 64
g = load(case)
p = g["p"]
sig = torch.from_numpy(g["signal"]).cuda()
ref = engine.compress_device(sig, p["tile"], K, energy_thresh=p["thr"], keep_intermediates=True, search="f32")
torch.cuda.synchronize()
c32 = ref.cand.cpu().numpy().reshape(-1, K)
print("nd", ref.n_domains, "nr", ref.n_ranges)
for plan in [(-1, 1), (0, 1), (1000, 2), (1000, 5)]:
    call("fwav_debug_topk_plan", *plan)
    r = engine.compress_device(sig, p["tile"], K, energy_thresh=p["thr"], keep_intermediates=True)
    torch.cuda.synchronize()
    c = r.cand.cpu().numpy().reshape(-1, K)
    bad = np.nonzero(~np.all(c == c32, axis=1))[0]
    print(f"plan {plan}: {len(bad)} rows differ from f32; first {bad[:8]}; blocks {np.unique(bad // 256)[:12]}")
    for q in bad[:2]:
        print("   q", q, "missing", sorted(set(c32[q]) - set(c[q]))[:6], "extra", sorted(set(c[q]) - set(c32[q]))[:6],
              "n(-1)", int((c[q] < 0).sum()))
call("fwav_debug_topk_plan", -1, 1)
