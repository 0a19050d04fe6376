#!/bin/bash
# session 18: single-launch tail at HEAD: share curve and per-tile timeline (RG_TILE_TIMES)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s18
timeout -k 10 200 python scripts/tail_probe.py curve > gpurun_out/s18/curve.json 2> gpurun_out/s18/curve.err
RAINGUN_HIP_LIB=$PWD/abvar/tt/libraingun_hip.so timeout -k 10 200 python scripts/tail_probe.py timeline > gpurun_out/s18/timeline.json 2> gpurun_out/s18/timeline.err
cat gpurun_out/s18/curve.json gpurun_out/s18/timeline.json
