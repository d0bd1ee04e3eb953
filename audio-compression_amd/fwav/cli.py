"""Command line, same sub-commands / flags / output naming as the reference (fractal.py:1550-1669).

  python fractal.py compress IN OUT [--tile 1024] [--energy-thresh 1e-4] [--gpu] [--batch] [--out DIR] [--workers 4]
  python fractal.py decompress IN [--out PATH] [--iter 8] [--eps 1e-3] [--gpu] [--batch] [--workers 4]

Non-batch OUTPUT / --out are used as directories (quirk Q8, fractal.py:1509, 1538).  Batch mode skips
files whose output exists and writes compression_metrics.json / decompression_metrics.json.  The reference's
file-level Pool (fractal.py:1596-1600, 1640-1644) becomes one worker process per GPU (at most --workers of them):
each worker is pinned to its own device at start-up and takes files from the shared queue, so a node's GPUs work
on different files at once.  Workers are started with 'spawn' (never fork after HIP initialisation).
"""
from __future__ import annotations

import argparse
import json
import logging
import multiprocessing as mp
import os

logger = logging.getLogger("fwavc")


def _compress_job(args):
    from .api import process_file_compress
    return process_file_compress(*args)


def _decompress_job(args):
    from .api import process_file_decompress
    return process_file_decompress(*args)


def _pin_device(counter, n_gpus):
    """Pool initializer: worker k of the pool takes GPU k (one process per GPU)."""
    with counter.get_lock():
        k = counter.value
        counter.value += 1
    if n_gpus > 0:
        import torch
        torch.cuda.set_device(k % n_gpus)


def _gpu_count() -> int:
    """Visible GPUs, counted without initialising HIP in this (parent) process."""
    try:
        import torch
        return int(torch.cuda.device_count())
    except Exception:  # noqa: BLE001
        return 0


def _run_pool(job, argsets, workers):
    """One worker process per GPU (at most `workers`), each pinned to its device; files are handed out one at a
    time in input order and the results come back in that order."""
    if not argsets:
        return []
    n_gpus = _gpu_count()
    procs = max(1, min(workers, len(argsets), n_gpus if n_gpus > 0 else workers))
    ctx = mp.get_context("spawn")
    counter = ctx.Value("i", 0)
    with ctx.Pool(processes=procs, initializer=_pin_device, initargs=(counter, n_gpus)) as pool:
        return pool.map(job, argsets, chunksize=1)


def main(argv=None):
    parser = argparse.ArgumentParser(description="Fractal WAV compressor with GPU, batch processing, and metrics")
    sub = parser.add_subparsers(dest="cmd")
    pc = sub.add_parser("compress")
    pc.add_argument("input", help="input WAV file or directory")
    pc.add_argument("output", nargs="?", default=None, help="output FWAV file (required unless --batch)")
    pc.add_argument("--tile", type=int, default=1024)
    pc.add_argument("--out", default=None, help="output directory (batch mode)")
    pc.add_argument("--energy-thresh", type=float, default=1e-4)
    pc.add_argument("--gpu", action="store_true")
    pc.add_argument("--batch", action="store_true", help="treat input as directory and compress all WAV inside")
    pc.add_argument("--workers", type=int, default=4, help="parallel file-level workers for batch")
    pd = sub.add_parser("decompress")
    pd.add_argument("input", help="input file or directory")
    pd.add_argument("--out", default=None, help="output file or directory")
    pd.add_argument("--iter", type=int, default=8)
    pd.add_argument("--eps", type=float, default=1e-3)
    pd.add_argument("--gpu", action="store_true")
    pd.add_argument("--batch", action="store_true", help="treat input as directory and decompress all FWAV inside")
    pd.add_argument("--workers", type=int, default=4, help="parallel file-level workers for batch")
    args = parser.parse_args(argv)

    if args.cmd == "compress":
        if not args.batch:
            if args.output is None:
                parser.error("compress requires OUTPUT unless --batch is used")
            return _compress_job((args.input, args.output, args.tile, args.energy_thresh, args.gpu))
        if args.output is not None:
            parser.error("Do not provide positional OUTPUT when using --batch; use --out instead")
        out_dir = args.out or args.input
        files = [os.path.join(args.input, f) for f in os.listdir(args.input) if f.lower().endswith(".wav")]
        todo = [f for f in files if not os.path.exists(os.path.join(out_dir, os.path.basename(f) + ".fwav"))]
        logger.info(f"Batch compressing {len(todo)}/{len(files)} files using {args.workers} workers")
        if not todo:
            logger.info("No files to compress — all already exist.")
            return None
        results = _run_pool(_compress_job, [(f, os.path.join(out_dir, os.path.basename(f) + ".fwav"), args.tile,
                                             args.energy_thresh, args.gpu) for f in todo], args.workers)
        metrics_file = os.path.join(out_dir, "compression_metrics.json")
        os.makedirs(os.path.dirname(metrics_file) or ".", exist_ok=True)
        with open(metrics_file, "w") as mf:
            json.dump(results, mf, indent=2)
        logger.info(f"Wrote metrics to {metrics_file}")
        return results
    if args.cmd == "decompress":
        if not args.batch:
            out_file = args.out or (os.path.splitext(args.input)[0] + "_recon.wav")
            return _decompress_job((args.input, out_file, args.iter, args.eps, args.gpu))
        out_dir = args.out or args.input
        files = [os.path.join(args.input, f) for f in os.listdir(args.input) if f.lower().endswith(".fwav")]
        todo = [f for f in files
                if not os.path.exists(os.path.join(out_dir, os.path.basename(f).replace(".fwav", "_recon.wav")))]
        logger.info(f"Batch decompressing {len(todo)}/{len(files)} files using {args.workers} workers")
        if not todo:
            logger.info("No files to decompress — all already exist.")
            return None
        results = _run_pool(_decompress_job, [(f, os.path.join(out_dir, os.path.basename(f).replace(".fwav", "_recon.wav")),
                                               args.iter, args.eps, args.gpu) for f in todo], args.workers)
        metrics_file = os.path.join(out_dir, "decompression_metrics.json")
        os.makedirs(os.path.dirname(metrics_file) or ".", exist_ok=True)
        with open(metrics_file, "w") as mf:
            json.dump(results, mf, indent=2)
        logger.info(f"Wrote metrics to {metrics_file}")
        return results
    parser.print_help()
    return None
