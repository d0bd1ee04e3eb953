#!/usr/bin/env bash
# SQ issue counters of the search kernel (cfg2, product geometry): two PMC passes of tools/topk_once.py
set -euo pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/sq
timeout -s KILL 120 rocprofv3 -L > gpurun_out/sq/list.txt 2>&1 || true
pass() {  # name counters...
  local name=$1; shift
  local have=()
  for c in "$@"; do grep -qw "$c" gpurun_out/sq/list.txt && have+=("$c") || echo "absent: $c"; done
  echo "pass $name: ${have[*]}"
  timeout -s KILL 150 rocprofv3 --pmc "${have[@]}" --kernel-trace --output-format csv -d gpurun_out/sq/$name -- python3 tools/topk_once.py 0 > gpurun_out/sq/$name.log 2>&1
}
pass p1 SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
pass p2 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
pass p3 SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES
echo done
