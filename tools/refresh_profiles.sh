#!/usr/bin/env bash
# GPU-box script: GPU tests, the default bench line, the rocprofv3 kernel-stats run of the same bench and the two
# HBM PMC passes (FETCH_SIZE / WRITE_SIZE in separate runs). Everything lands in gpurun_out/; summarise with
#   tools/prof_summary.py gpurun_out/prof/run_results.db --csv profiles/rNN_kernel_stats_cfg2.csv
#   tools/pmc_summary.py --fetch gpurun_out/pmc_fetch --write gpurun_out/pmc_write --config cfg2 --out profiles/pmc_cfg2.json
# Each GPU step has its own time limit; the script stops at the first failing step.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() {  # name seconds command...
  local name=$1 secs=$2
  shift 2
  echo "=== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1 || { echo "step $name failed: $?"; tail -20 "gpurun_out/$name.log"; exit 1; }
  tail -3 "gpurun_out/$name.log"
}
step gputests 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step bench 400 python -u bench.py
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
step prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -- python3 bench.py --no-cpu-baseline --steps 2 --warmup 1
find gpurun_out/prof -name "*.db" | head -3
