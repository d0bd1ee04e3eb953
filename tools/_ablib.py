"""Tools only: make fwav._lib use an experiment build (tools/ab_build.sh) instead of the product library.  Experiment
builds carry no source digest, so the product loader's provenance check (fwav._lib.lib) is bypassed here on purpose."""
import ctypes as C
import os


def use(path: str) -> None:
    from fwav import _lib
    dll = C.CDLL(os.path.abspath(path))
    for name, (res, args) in {**_lib.SIGNATURES, **_lib.DEBUG_SIGNATURES}.items():
        fn = getattr(dll, name, None)
        if fn is not None:
            fn.restype, fn.argtypes = res, args
    _lib.LIB_PATH = os.path.abspath(path)
    _lib._libs["product"] = _lib._libs["debug"] = dll
