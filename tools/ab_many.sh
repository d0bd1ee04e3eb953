#!/bin/bash
# Several tools/ab_topk.py runs in one GPU call, each under its own time limit; stops at the first failure.
# usage: tools/ab_many.sh OUT_PREFIX "ENV=.. ENV=..|lib1 lib2 .." ...   -> gpurun_out/OUT_PREFIX_<i>.log
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
pre=$1; shift
i=0
for spec in "$@"; do
  envs=${spec%%|*}; libs=${spec#*|}
  log=gpurun_out/${pre}_$i.log
  echo "== $envs :: $libs" | tee "$log"
  env $envs timeout -k 10 300 python3 -u tools/ab_topk.py $libs >> "$log" 2>&1
  rc=$?
  grep -E "median|overflowed" "$log" || true
  if [ $rc -ne 0 ]; then echo "run $i failed rc=$rc"; tail -20 "$log"; exit $rc; fi
  i=$((i+1))
done
