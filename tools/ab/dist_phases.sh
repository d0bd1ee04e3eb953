#!/usr/bin/env bash
# GPU-box script: the sharded bench path's collectives on one GPU — world size 1 over RCCL (FWAV_BENCH_FORCE_DIST),
# then two gloo ranks sharing cuda:0 — for the broadcast / compute / gather phases of its untimed phase steps.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
FWAV_BENCH_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 1 --steps 10 --warmup 3 --no-cpu-baseline --no-extras \
  > gpurun_out/dist_world1_rccl.log 2>&1
FWAV_BENCH_BACKEND=gloo FWAV_BENCH_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --steps 10 --warmup 3 \
  --no-cpu-baseline --no-extras > gpurun_out/dist_world2_gloo_shared.log 2>&1
for f in dist_world1_rccl dist_world2_gloo_shared; do
  python - "$f" <<'PY'
import json, sys
l = [x for x in open(f"gpurun_out/{sys.argv[1]}.log") if x.startswith("{")][-1]
d = json.loads(l)
print(sys.argv[1], "ms/step", round(d["ms_per_step"], 3), "streams", d["config"].get("streams"))
for r in d.get("per_rank", []):
    print("   ", {k: round(v, 3) for k, v in r.items()})
PY
done
