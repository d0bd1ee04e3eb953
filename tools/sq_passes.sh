#!/usr/bin/env bash
# SQ counter passes over the similarity search (tools/topk_once.py), one rocprofv3 --pmc run per dbg value.
# usage: tools/sq_passes.sh "COUNTERS" dbg [dbg ...]   -> gpurun_out/sq_<dbg>/ (CSV), summary on stdout
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
counters=$1; shift
for d in "$@"; do
  out=gpurun_out/sq_$d
  rm -rf "$out"
  timeout -s KILL 120 rocprofv3 --pmc $counters --kernel-trace --output-format csv -d "$out" -- python3 tools/topk_once.py "$d" > "$out.log" 2>&1
  python3 tools/sq_summary.py "$out" "$d"
done
