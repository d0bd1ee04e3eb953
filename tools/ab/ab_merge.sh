#!/usr/bin/env bash
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
N=audio-compression_amd/fwav/libfwav_debug.so
B=tools/ab/libfwav_base.so
tools/gpu_steps.sh \
 "ab_cfg2:300:python -u tools/lib_ab.py $B $N 9" \
 "ab_eighth:300:AB_NQ=41344 python -u tools/lib_ab.py $B $N 15" \
 "prof_new:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_new -o run -- python3 tools/lib_ab.py $N $N 5" \
 "prof_base:300:rocprofv3 --kernel-trace --stats -d gpurun_out/prof_base -o run -- python3 tools/lib_ab.py $B $B 5" \
 "tests:900:python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_cfg2_tuples.py tests/test_gpu_floor.py tests/test_gpu_oracle_rows.py tests/test_gpu_parity.py"
