"""Summarise one rocprofv3 --pmc CSV directory for k_sim_topk_f16 (last dispatch): counters and derived ratios.
usage: python tools/sq_summary.py DIR LABEL"""
import csv
import glob
import os
import sys

d, label = sys.argv[1], sys.argv[2]
rows = {}
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    with open(f, newline="") as fh:
        for r in csv.DictReader(fh):
            if "k_sim_topk_f16" not in r["Kernel_Name"]:
                continue
            rows.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
last = rows[max(rows)]
print(label, " ".join(f"{k}={v:.4g}" for k, v in sorted(last.items())))
wc = last.get("SQ_WAVE_CYCLES")
if wc:
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
        if k in last:
            print(f"  {k}/WAVE_CYCLES = {last[k] / wc:.3f}")
if "SQ_VALU_MFMA_BUSY_CYCLES" in last and "GRBM_GUI_ACTIVE" in last:
    # MFMA busy summed over SIMDs (cycles) vs 1024 SIMDs x kernel cycles
    print(f"  MFMA busy / (1024 SIMD x GUI_ACTIVE) = {last['SQ_VALU_MFMA_BUSY_CYCLES'] / (1024 * last['GRBM_GUI_ACTIVE']):.3f}")
