"""fwav — MI355X-native fractal WAV compression engine (drop-in for xavenordu/Audio-Compression's fractal.py).

Hot path on the GPU through the C-ABI library ``libfwav.so`` (HIP, gfx950); see DESIGN.md.  Importing the package
imports neither torch nor the device pipeline: ``fwav.hipctypes`` (the torch-free binding) needs only numpy.
"""
from .matches import MatchList  # noqa: F401


def geometry(tile_size: int) -> tuple[int, int]:
    """range_size, domain_step (fractal.py:1070-1071)."""
    rs = max(4, tile_size // 256)
    return rs, max(1, rs // 4)


__all__ = ["geometry", "MatchList"]
