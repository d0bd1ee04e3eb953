#!/usr/bin/env bash
# GPU-box script: one rank's pipelined sharded compress (tools/shard_step.py) with consecutive calls spread over
# 1, 2 and 3 HIP streams, at N = 1 and every rank of N = 8.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for s in 1 2 3; do
  echo "=== streams $s"
  timeout -k 10 400 python -u tools/shard_step.py --steps 30 --ns 1,8 --streams $s --lags 3,4,6 > gpurun_out/streams_$s.log 2>&1 \
    || { echo "streams $s failed: $?"; tail -20 gpurun_out/streams_$s.log; exit 1; }
  tail -n 1 gpurun_out/streams_$s.log
done
