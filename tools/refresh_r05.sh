#!/usr/bin/env bash
# GPU-box script (round 5): the default bench line, the rocprofv3 kernel-stats run of the same bench command, and
# the two HBM PMC passes (FETCH_SIZE / WRITE_SIZE, separate runs).  Each step has its own time limit; the script
# stops at the first failing step.  Summaries: tools/prof_summary.py, tools/pmc_summary.py.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
step() {  # name seconds command...
  local name=$1 secs=$2
  shift 2
  echo "=== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1 || { echo "step $name failed: $?"; tail -20 "gpurun_out/$name.log"; exit 1; }
  tail -c 400 "gpurun_out/$name.log"; echo
}
rm -rf gpurun_out/prof_r05 gpurun_out/pmc_fetch_r05 gpurun_out/pmc_write_r05
step bench_r05 500 python -u bench.py --steps 20 --warmup 5
step prof_r05 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r05 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline
step pmc_fetch_r05 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_r05 -- python3 bench.py --no-cpu-baseline --no-extras --steps 2 --warmup 1
step pmc_write_r05 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write_r05 -- python3 bench.py --no-cpu-baseline --no-extras --steps 2 --warmup 1
step shard_step_r05 600 python -u tools/shard_step.py --steps 20
step shard_step2_r05 400 python -u tools/shard_step.py --steps 20 --ns 1,8 --ranks 0,3,7 --streams 2 --lags 3,4
# SQ issue counters of the search's first pass (product geometry), three PMC passes (tools/sq_summary.py --json)
rm -rf gpurun_out/sq
bash tools/ab/sq_pmc.sh
