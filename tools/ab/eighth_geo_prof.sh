#!/usr/bin/env bash
# GPU-box script (round 6): one rank's eighth of cfg2 (AB_NQ queries, default 41,344, the last block) under floor x
# geometry settings (tools/diag/topk_reps.py, debug library), one rocprofv3 kernel trace each: the launch sequence of
# one call is read back with tools/prof_timeline.py.  Settings "floor|geometry|p2" (floor: FWAV_DEBUG_TOPK_FLOOR,
# "-" = unset; geometry: FWAV_DEBUG_TOPK_GEOMETRY, "-" = the product's choice).
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
NQ=${AB_NQ:-41344}
SETTINGS=${AB_SETTINGS:-"0|-|0 2:10|2|0 0|2|0 2:3|2|0"}
a=()
for v in $SETTINGS; do
  IFS='|' read -r f g p2 <<< "$v"
  n="eg_${NQ}${AB_LO:+_lo$AB_LO}_f${f//:/_}_g${g}_p${p2}"
  env=""
  [ "$f" != "-" ] && env+="FWAV_DEBUG_TOPK_FLOOR=$f "
  [ "$g" != "-" ] && env+="FWAV_DEBUG_TOPK_GEOMETRY=$g "
  rm -rf "gpurun_out/$n"
  a+=("$n:300:AB_NQ=$NQ ${AB_LO:+AB_LO=$AB_LO }${env}FWAV_DEBUG_TOPK_P2=$p2 rocprofv3 --kernel-trace --stats -d gpurun_out/$n -o run -- python3 tools/diag/topk_reps.py 15")
done
tools/gpu_steps.sh "${a[@]}"
