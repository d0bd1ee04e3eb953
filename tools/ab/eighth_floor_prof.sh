#!/usr/bin/env bash
# GPU-box script (round 6): kernel-level breakdown of one rank's eighth of cfg2 (41,344 queries, the last block) under
# floor settings (tools/diag/topk_reps.py, debug library): off, and forced on with the pilots' rank 10 / 5 / 3 (second
# pass pieces by size: 32 below 131,072 queries); then same-process A/Bs against the previous library.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
a=()
for v in "0:0" "2:10:0" "2:5:0" "2:3:0" "0:0"; do
  p2=${v##*:}; f=${v%:*}
  n="ef_${f//:/_}_p${p2}"
  rm -rf "gpurun_out/$n"
  a+=("$n:300:AB_NQ=41344 FWAV_DEBUG_TOPK_FLOOR=$f FWAV_DEBUG_TOPK_P2=$p2 rocprofv3 --kernel-trace --stats -d gpurun_out/$n -o run -- python3 tools/diag/topk_reps.py 15")
done
B=${AB_BASE:-tools/ab/libfwav_prev.so}
N=audio-compression_amd/fwav/libfwav_debug.so
tools/gpu_steps.sh "${a[@]}" \
 "ab_cfg2:300:python -u tools/lib_ab.py $B $N 9" \
 "ab_quarter:300:AB_NQ=82688 python -u tools/lib_ab.py $B $N 11"
