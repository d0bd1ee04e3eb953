"""Issue-level summary of the search kernel's SQ counters (rocprofv3 --pmc CSV passes of tools/topk_once.py, made by
tools/ab/sq_pmc.sh): per dispatch of k_sim_topk_f16's first pass, the shares of wave time (active / issue-stalled /
parked), instruction counts per level-1 tile and per MFMA, and pipe utilisation per SIMD (SQ_* quad-cycle counters
×4; SQ_VALU_MFMA_BUSY_CYCLES in cycles; kernel cycles = GRBM_GUI_ACTIVE / 8 XCDs).
usage: python tools/sq_summary.py gpurun_out/sq [--tiles N] [--json profiles/sq_cfg2.json --config cfg2]
(--json: the executed-MFMA figures bench.py puts beside its algorithmic roofline)"""
import argparse
import collections
import json
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
        # the newest pass file (gpurun merges each call's files into the same directory)
        for r in csv.DictReader(open(max(fs, key=os.path.getmtime))):
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
    ap.add_argument("--json", default=None, help="write the executed-MFMA summary bench.py reads")
    ap.add_argument("--config", default="cfg2")
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
    if a.json:
        # every MFMA of the search is v_mfma_f32_32x32x16_f16: 2·32·32·16 = 32,768 flop per wave instruction
        d = {"config": a.config, "kernel": "k_sim_topk_f16 (first pass)",
             "sq_insts_mfma_per_launch": c.get("SQ_INSTS_MFMA"),
             "mfma_executed_flop_per_launch": c["SQ_INSTS_MFMA"] * 32768 if "SQ_INSTS_MFMA" in c else None,
             "mfma_busy_frac": (c["SQ_VALU_MFMA_BUSY_CYCLES"] / SIMDS / cyc) if "SQ_VALU_MFMA_BUSY_CYCLES" in c
             else None,
             "kernel_cycles": cyc, "kernel_ms_at_2p4ghz": cyc / 2.4e6,
             "wave_time": {"active": c["SQ_ACTIVE_INST_ANY"] / wc, "issue_stalled": c["SQ_WAIT_INST_ANY"] / wc,
                           "parked": c["SQ_WAIT_ANY"] / wc},
             "source": f"rocprofv3 --pmc SQ passes of tools/topk_once.py ({a.root})"}
        with open(a.json, "w") as f:
            json.dump(d, f, indent=1)
        print(f"wrote {a.json}")


if __name__ == "__main__":
    main()
