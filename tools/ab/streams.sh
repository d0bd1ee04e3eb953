#!/usr/bin/env bash
# GPU-box script: one rank's pipelined sharded compress (tools/shard_step.py) with consecutive calls spread over
# 1 and 2 HIP streams, at N = 1 and the ranks of N = 8 (${RANKS:-all}).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for s in ${STREAMS:-1 2}; do
  echo "=== streams $s"
  timeout -k 10 400 python -u tools/shard_step.py --steps 30 --ns ${NS:-1,8} --ranks "${RANKS:-}" --streams $s --lags ${LAGS:-3,4,6} > gpurun_out/streams_$s.log 2>&1 \
    || { echo "streams $s failed: $?"; tail -20 gpurun_out/streams_$s.log; exit 1; }
  tail -n 1 gpurun_out/streams_$s.log
done
