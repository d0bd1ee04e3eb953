#!/usr/bin/env bash
# GPU-box script (round 4): the default bench line, the rocprofv3 kernel-stats run of the same bench command, and
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
rm -rf gpurun_out/prof_r04 gpurun_out/pmc_fetch_r04 gpurun_out/pmc_write_r04
step bench_r04 500 python -u bench.py --steps 20 --warmup 5
step prof_r04 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r04 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline
step pmc_fetch_r04 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_r04 -- python3 bench.py --no-cpu-baseline --no-extras --steps 2 --warmup 1
step pmc_write_r04 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write_r04 -- python3 bench.py --no-cpu-baseline --no-extras --steps 2 --warmup 1
step shard_step_r04 600 python -u tools/shard_step.py --steps 20
