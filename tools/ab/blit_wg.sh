#!/usr/bin/env bash
# GPU-box script (round 6): the cfg2 bench (two streams) with the HIP runtime's blit-copy kernels limited to 16
# workgroups (DEBUG_CLR_LIMIT_BLIT_WG) against the default, alternating; then the parity tests of this tree.
set -u
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
a=()
for i in 1 2; do
  a+=("bench_def_$i:300:python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extras"
      "bench_blit16_$i:300:DEBUG_CLR_LIMIT_BLIT_WG=16 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-extras")
done
tools/gpu_steps.sh "${a[@]}" \
 "tests:900:python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_cfg2_tuples.py tests/test_gpu_floor.py tests/test_gpu_parity.py tests/test_gpu_decode.py"
