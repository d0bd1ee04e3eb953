#!/usr/bin/env python3
"""HBM traffic per launch from two rocprofv3 counter passes (CSV output), gfx950-corrected.

MI355X_MICROARCH.md §HBM / cdna_hip_programming.md §7: FETCH_SIZE and WRITE_SIZE cannot share a pass
(TCC slots), both are in KiB, and on gfx950 FETCH_SIZE reports exactly half the bytes of a wide coalesced
streaming read, so   hbm_bytes = (2 · FETCH_SIZE + WRITE_SIZE) · 1024   per dispatch.

usage: tools/pmc_summary.py --fetch DIR --write DIR --config cfg2 --out profiles/pmc_cfg2.json
(bench.py reads profiles/pmc_<config>.json for the `traffic` of its own config only)
DIR = the rocprofv3 -d directory of a `--pmc FETCH_SIZE` (resp. WRITE_SIZE) `--kernel-trace
--output-format csv` run; every *counter_collection.csv below it is read.
"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict

KEYS = {"k_sim_topk_f16": "sim_topk_hbm_bytes_per_launch", "k_affine": "affine_hbm_bytes_per_launch"}


def per_kernel(d, counter):
    vals = defaultdict(list)
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    # gpurun merges each call's gpurun_out/ into the local one, so older passes may lie beside this one: newest only
    files = [max(files, key=os.path.getmtime)]
    for f in files:
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                vals[row["Kernel_Name"]].append(float(row["Counter_Value"]))
    return vals


def short(name):
    base = name.split("(")[0]
    return base.replace("void ", "").strip()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--config", required=True, help="bench config the passes ran (cfg2, cfg3, ...)")
    ap.add_argument("--source", default="rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of bench.py")
    a = ap.parse_args()
    fe = per_kernel(a.fetch, "FETCH_SIZE")
    wr = per_kernel(a.write, "WRITE_SIZE")
    kernels = {}
    for k in sorted(set(fe) | set(wr)):
        f = sum(fe.get(k, [0.0])) / max(len(fe.get(k, [])), 1)
        w = sum(wr.get(k, [0.0])) / max(len(wr.get(k, [])), 1)
        kernels[short(k)] = {"dispatches": len(fe.get(k, [])), "fetch_kib_raw": f, "write_kib": w,
                             "hbm_bytes_per_launch": (2.0 * f + w) * 1024.0}
    out = {"formula": "(2*FETCH_SIZE + WRITE_SIZE)*1024 per dispatch (gfx950 FETCH_SIZE half-count correction)",
           "config": a.config, "source": a.source, "kernels": kernels}
    # per pattern: the dominant kernel of the bench's own steps (the PMC passes run with --no-extras) — the one that
    # moves the most bytes per dispatch: the search's first pass, not the floor's later passes or the overflow
    # relaunches that also match the pattern
    for pat, key in KEYS.items():
        cands = [(v["hbm_bytes_per_launch"], k) for k, v in kernels.items()
                 if pat in k and v["hbm_bytes_per_launch"] > 1e6]
        if cands:
            out[key] = max(cands)[0]
            out[key.replace("_bytes_per_launch", "_kernel")] = max(cands)[1]
    with open(a.out, "w") as fh:
        json.dump(out, fh, indent=1)
    for k, v in sorted(kernels.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"]):
        print(f"{k[:80]:80s} {v['hbm_bytes_per_launch'] / 1e6:12.2f} MB/launch  ({v['dispatches']} dispatches)")


if __name__ == "__main__":
    main()
