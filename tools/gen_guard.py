"""Rewrite the product-build guard of fwav_topk.hip / fwav_affine.hip from the knobs each file defines
(#ifndef / #ifdef FWAV_TOPK_* / FWAV_AFF_*), so that every knob stays refused without -DFWAV_DEBUG_API
(tests/test_capi.py::test_every_knob_is_guarded).  usage: python tools/gen_guard.py"""
import os
import re

ROOT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "audio-compression_amd", "csrc")
for f, pre in (("fwav_topk.hip", "FWAV_TOPK_"), ("fwav_affine.hip", "FWAV_AFF_")):
    path = os.path.join(ROOT, f)
    s = open(path).read()
    a = s.index("#if !defined(FWAV_DEBUG_API) && (")
    b = s.index("#error", a)
    knobs = sorted(set(re.findall(r"#ifn?def (" + pre + r"\w+)", s)))
    items = [f"defined({k})" for k in knobs]
    out, line = [], "#if !defined(FWAV_DEBUG_API) && ("
    for i, it in enumerate(items):
        piece = it + (" || " if i < len(items) - 1 else ")")
        if len(line) + len(piece.rstrip()) > 117:
            out.append(line.rstrip() + " \\")
            line = "    "
        line += piece
    out.append(line)
    s = s[:a] + "\n".join(out) + "\n" + s[b:]
    open(path, "w").write(s)
    print(f, len(knobs), "knobs")
