#!/usr/bin/env bash
# GPU-box script (round 6): one rank's eighth of cfg2 (N = 8), two streams, 4 calls in flight, with the speculative
# floor off (the default below 65,536 queries) and forced on (pilots' rank 10 / 5), base and centroid geometry; the
# cfg3 bench without the host tie ranking; the merge A/B.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1 FWAV_DEBUG_LIBRARY=1
a=()
for v in "-1:" "2:10:" "2:5:" "2:10:2"; do
  f=${v%:*}; g=${v##*:}
  n="eighth_f${f//:/_}_g${g:-d}"
  a+=("$n:400:FWAV_DEBUG_TOPK_FLOOR=$f ${g:+FWAV_DEBUG_TOPK_GEOMETRY=$g} python -u tools/shard_step.py --ns 8 --ranks 0,5 --streams 2 --lags 4 --steps 40")
done
tools/gpu_steps.sh "${a[@]}" \
 "ab_cfg2:300:python -u tools/lib_ab.py tools/ab/libfwav_base.so audio-compression_amd/fwav/libfwav_debug.so 9" \
 "cfg3_index:600:python -u bench.py --config cfg3 --steps 5 --warmup 2 --no-cpu-baseline --no-extras --tie-order index"
