#!/usr/bin/env bash
# GPU-box script: same-box A/B of the speculative floor through whole programs (the debug library, its floor knob set
# by FWAV_DEBUG_TOPK_FLOOR): bench.py at N = 1, then one rank's pipelined step at N = 8 on two streams.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1 FWAV_DEBUG_LIBRARY=1
mkdir -p gpurun_out
for f in 0 -1 0 -1; do
  FWAV_DEBUG_TOPK_FLOOR=$f timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-extras > gpurun_out/floor_bench_$f.log 2>&1
  python - "$f" <<'PY'
import json, sys
l = [x for x in open(f"gpurun_out/floor_bench_{sys.argv[1]}.log") if x.startswith("{")][-1]
d = json.loads(l)
print("bench floor", sys.argv[1], round(d["ms_per_step"], 3), "sim_topk", round(d["stage_ms"]["sim_topk"], 3))
PY
done
for f in 0 2:10; do
  FWAV_DEBUG_TOPK_FLOOR=$f timeout -k 10 300 python -u tools/shard_step.py --steps 30 --ns 8 --ranks 0,4 --streams 2 --lags 3,4 > "gpurun_out/floor_shard_${f/:/_}.log" 2>&1
  echo "shard floor $f"; grep '^8 ' "gpurun_out/floor_shard_${f/:/_}.log" | python -c "
import json,sys
d=json.loads(sys.stdin.read()[2:])
for r in d['ranks']: print('  rank', r['rank'], {k: round(v, 3) for k, v in r['wall_ms_pipelined_by_lag'].items()}, 'topk', round(r['stage_ms']['sim_topk'], 3))"
done
