"""Issue-level summary of the search kernel's SQ counters (rocprofv3 --pmc CSV passes of tools/topk_once.py, made by
tools/ab/sq_pmc.sh): per dispatch of k_sim_topk_f16's first pass, the shares of wave time (active / issue-stalled /
parked), instruction counts per level-1 tile and per MFMA, and pipe utilisation per SIMD (SQ_* quad-cycle counters
×4; SQ_VALU_MFMA_BUSY_CYCLES in cycles; kernel cycles = GRBM_GUI_ACTIVE / 8 XCDs).
usage: python tools/sq_summary.py gpurun_out/sq [--tiles N]"""
import argparse
import collections
import csv
import glob
import os

SIMDS = 256 * 4


def load(root):
    out = collections.defaultdict(dict)  # pass -> {counter: value} for the largest topk dispatch
    for d in sorted(glob.glob(os.path.join(root, "p*"))):
        fs = glob.glob(os.path.join(d, "runc", "*_counter_collection.csv"))
        if not fs:
            continue
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        for r in csv.DictReader(open(fs[0])):
            if "sim_topk" in r["Kernel_Name"]:
                per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
        if per:  # the last big dispatch (the timed repetition)
            best = max(per.values(), key=lambda v: max(v.values()))
            out[os.path.basename(d)] = dict(best)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--tiles", type=float, default=646 * 8 * 41312,
                    help="level-1 tiles of one launch (cfg2: 646 blocks × 8 waves × 41,312 tiles)")
    a = ap.parse_args()
    c = {}
    for v in load(a.root).values():
        c.update(v)
    cyc = c["GRBM_GUI_ACTIVE"] / 8
    wc = c["SQ_WAVE_CYCLES"]
    print(f"kernel cycles {cyc:.3e}; waves resident per SIMD {wc * 4 / SIMDS / cyc:.2f}")
    print("wave time: active {:.1%}  issue-stalled {:.1%}  parked (waitcnt/barrier) {:.1%}".format(
        c["SQ_ACTIVE_INST_ANY"] / wc, c["SQ_WAIT_INST_ANY"] / wc, c["SQ_WAIT_ANY"] / wc))
    for k in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_MISC",
              "SQ_ACTIVE_INST_FLAT", "SQ_LDS_IDX_ACTIVE"):
        if k in c:
            print(f"{k:28s} {c[k] * 4 / SIMDS / cyc:6.1%} of SIMD cycles")
    if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
        print(f"{'MFMA busy':28s} {c['SQ_VALU_MFMA_BUSY_CYCLES'] / SIMDS / cyc:6.1%} of SIMD cycles")
    t = a.tiles
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_VMEM", "SQ_INSTS_BRANCH"):
        if k in c:
            print(f"{k:28s} {c[k]:.3e}  = {c[k] / t:5.2f} per level-1 tile")


if __name__ == "__main__":
    main()
