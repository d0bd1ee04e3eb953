#!/usr/bin/env bash
# Run named GPU steps with their own time limits; stop the call at the first fault/abort/timeout
# (exit codes other than 0 and 1), continue past ordinary failures (exit 1 = failed tests/assertion).
# usage: tools/gpu_steps.sh "name:seconds:command" ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== $name (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name rc=$rc ($(( $(date +%s) - start ))s)"
  tail -n 15 "gpurun_out/$name.log"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then
    echo "stopping: $name exited $rc"; exit "$rc"
  fi
done
