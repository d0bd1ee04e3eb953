#!/usr/bin/env bash
# GPU-box script (round 6): the default bench line (cfg2, two streams), the rocprofv3 kernel-stats run of the same
# bench command, the two HBM PMC passes (FETCH_SIZE / WRITE_SIZE, separate runs), the cfg3 bench, the merge's inputs
# and the strong-scaling projection (every N on two streams).  Each step has its own time limit (tools/gpu_steps.sh:
# a fault, abort or time limit ends the call).  Summaries: tools/prof_summary.py, tools/pmc_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
rm -rf gpurun_out/prof_r06 gpurun_out/pmc_fetch_r06 gpurun_out/pmc_write_r06
STEPS=${REFRESH_STEPS:-"merge_inputs bench prof pmc cfg3 shard"}
args=()
for s in $STEPS; do
  case $s in
    merge_inputs) args+=("merge_inputs_r06:200:python -u tools/diag/merge_inputs.py") ;;
    bench) args+=("bench_r06:600:python -u bench.py --steps 20 --warmup 5") ;;
    prof) args+=("prof_r06:500:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r06 -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --streams 1") ;;
    pmc) args+=("pmc_fetch_r06:300:rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch_r06 -- python3 bench.py --no-cpu-baseline --no-extras --steps 2 --warmup 1"
                "pmc_write_r06:300:rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write_r06 -- python3 bench.py --no-cpu-baseline --no-extras --steps 2 --warmup 1") ;;
    cfg3) args+=("bench_cfg3_r06:600:python -u bench.py --config cfg3 --steps 5 --warmup 2 --no-cpu-baseline --no-extras") ;;
    shard) args+=("shard_step_r06:900:python -u tools/shard_step.py --steps 20 --streams 2 --lags 4") ;;
  esac
done
tools/gpu_steps.sh "${args[@]}"
