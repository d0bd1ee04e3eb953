#!/bin/bash
# Kernel times of the search (first pass + k_merge_pieces) at cfg2 and at one rank's eighth, and SQ counters of
# the merge kernel (one --pmc pass each).  -> gpurun_out/pm/
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/pm
run() {  # name env... -- cmd
  local name=$1; shift
  timeout -s KILL 150 env "$@" > gpurun_out/pm/$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/pm/$name.log; exit 1; }
}
run stats_cfg2 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pm/stats_cfg2 -- python3 tools/topk_once.py 0
run stats_eighth AB_NQ=41344 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pm/stats_eighth -- python3 tools/topk_once.py 0
run sq_cfg2 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_INSTS_SALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pm/sq_cfg2 -- python3 tools/topk_once.py 0
for d in stats_cfg2 stats_eighth; do echo "== $d"; f=$(find gpurun_out/pm/$d -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f" | head -8; done
f=$(find gpurun_out/pm/sq_cfg2 -name "*counter_collection.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(sys.argv[1])):
    if "merge" in r["Kernel_Name"] or "sim_topk" in r["Kernel_Name"]:
        agg[(r["Kernel_Name"][:60], r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in agg.items():
    print(k, {a: f"{b:.3e}" for a, b in v.items()})
PY
