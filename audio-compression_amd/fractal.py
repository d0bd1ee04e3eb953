"""Drop-in ``fractal`` module: the public surface of xavenordu/Audio-Compression's ``fractal.py`` on the
MI355X engine (``from fractal import compress_audio, save_compressed, load_compressed, decompress_audio,
compute_snr`` as in the reference's test_e2e.py:3).

Module global ``top_k`` (fractal.py:77) is honoured exactly as the reference does when ``compress_audio``
is called without ``top_k=``.
"""
import logging

from fwav.api import (EMBED_K, FWAV_VERSION, compress_audio, compute_snr, decompress_audio,  # noqa: F401
                      process_file_compress, process_file_decompress)
from fwav.cli import main  # noqa: F401
from fwav.fwavio import load_compressed, read_wav_mono, save_compressed, write_wav  # noqa: F401
from fwav.matches import MatchList  # noqa: F401

logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s: %(message)s")
logger = logging.getLogger("fwavc")

top_k = 32  # number of candidates to consider per range (fractal.py:77)

if __name__ == "__main__":
    main()
