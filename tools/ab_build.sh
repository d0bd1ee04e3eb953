#!/bin/bash
# Build a variant of libfwav with extra -D flags for tools/ab_topk.py.
# usage: tools/ab_build.sh NAME [-DFWAV_TOPK_W=4 -DFWAV_TOPK_QS=2 ...]   ->  tools/ab/libfwav_NAME.so
set -euo pipefail
cd "$(dirname "$0")/.."
name=$1
shift
out=tools/ab/obj_$name
mkdir -p "$out"
flags=(--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -DFWAV_DEBUG_API "$@")
pids=()
for s in audio-compression_amd/csrc/*.hip; do
  hipcc "${flags[@]}" -c "$s" -o "$out/$(basename "$s" .hip).o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
hipcc --offload-arch=gfx950 -shared -fPIC "$out"/*.o -o "tools/ab/libfwav_$name.so"
rm -rf "$out"
echo "tools/ab/libfwav_$name.so"
