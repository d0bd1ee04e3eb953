"""fwav — MI355X-native fractal WAV compression engine (drop-in for xavenordu/Audio-Compression's fractal.py).

Hot path on the GPU through the C-ABI library ``libfwav.so`` (HIP, gfx950); see DESIGN.md.
"""
from .engine import geometry  # noqa: F401
from .matches import MatchList  # noqa: F401

__all__ = ["geometry", "MatchList"]
