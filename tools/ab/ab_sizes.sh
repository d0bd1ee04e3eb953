#!/usr/bin/env bash
# GPU-box script (round 6): same-process A/B of the search (previous library vs this tree's debug library) at the
# rank shares of cfg2 (N = 1, 2, 4, 8), then the search's parity tests.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
B=${AB_BASE:-tools/ab/libfwav_prev.so}
N=${AB_NEW:-audio-compression_amd/fwav/libfwav_debug.so}
tools/gpu_steps.sh \
 "ab_n1:300:python -u tools/lib_ab.py $B $N 9" \
 "ab_n2:300:AB_NQ=165375 python -u tools/lib_ab.py $B $N 11" \
 "ab_n4:300:AB_NQ=82688 python -u tools/lib_ab.py $B $N 13" \
 "ab_n8:300:AB_NQ=41344 python -u tools/lib_ab.py $B $N 15" \
 ${AB_TESTS:+"tests:900:python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_cfg2_tuples.py tests/test_gpu_floor.py tests/test_gpu_parity.py"}
