#!/usr/bin/env bash
# GPU-box script: same-process A/B of the search (base library vs this tree's debug library) at cfg2 and one rank's
# eighth, and rocprofv3 kernel stats of this tree's search.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
N=audio-compression_amd/fwav/libfwav_debug.so
B=${AB_BASE:-tools/ab/libfwav_base.so}
tools/gpu_steps.sh \
 "ab_cfg2:300:python -u tools/lib_ab.py $B $N 9" \
 "ab_eighth:300:AB_NQ=41344 python -u tools/lib_ab.py $B $N 15" \
 "prof_new:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_new -o run -- python3 tools/lib_ab.py $N $N 5"
