"""Build provenance of ``libfwav.so`` (no torch import: ``__graft_entry__.build`` loads this file directly).

The library embeds the SHA-256 of the sources it was compiled from and of the compiler flags
(``fwav_build_digest()``); ``build()`` rebuilds whenever the digest of the sources beside it differs, and
``fwav._lib.lib()`` refuses to bind a library whose digest does not match them — so a prebuilt binary that was not
built from the committed sources can never run the product path or the tests.
"""
from __future__ import annotations

import glob
import hashlib
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(_HERE)
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")

HIPCC_FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
               "-fhip-fp32-correctly-rounded-divide-sqrt", "-Wall", "-Wno-unused-result"]


def sources() -> list[str]:
    """Every file libfwav.so depends on: the HIP sources, their private headers and the public C-ABI header."""
    return (sorted(glob.glob(os.path.join(CSRC, "*.hip"))) + sorted(glob.glob(os.path.join(CSRC, "*.h")))
            + sorted(glob.glob(os.path.join(ROOT, "include", "*.h"))))


def source_digest() -> str | None:
    """SHA-256 over the compiler flags and every source (relative path + bytes); None when the sources are absent."""
    srcs = sources()
    if not any(s.endswith(".hip") for s in srcs):
        return None
    h = hashlib.sha256()
    h.update("\0".join(HIPCC_FLAGS).encode())
    for s in srcs:
        h.update(b"\0" + os.path.relpath(s, ROOT).encode() + b"\0")
        with open(s, "rb") as f:
            h.update(f.read())
    return h.hexdigest()
