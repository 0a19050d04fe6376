#!/bin/bash
# session 28: north-star single launches against the per-lane walk depth (rg_debug_set_lane_depth)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s28
for ld in 1 0 2 99 1; do
  timeout -k 10 300 python scripts/latency_probe.py --no-multi --lane-depth=$ld synth1024 > gpurun_out/s28/lat_ld$ld.json 2> gpurun_out/s28/lat_ld$ld.err
  python -c "import json,sys; d=json.load(open(sys.argv[1]))['synth1024']; print('lane_depth', sys.argv[2], 'whole', d['whole_kernel_ms'], 'share8', d['share8_kernel_ms'], 'max', d['share8_max_ms'])" gpurun_out/s28/lat_ld$ld.json $ld
done
