#!/bin/bash
# Round-5 session 8: light-buffer resolution -- cube-map cells per face edge 64 / 128 (in-tree) /
# 256, directional cell edge 0.25 / 0.5 (in-tree) / 1.0 mean radii; north star and the configs[4]
# scene at 1080p, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L="raingun_amd/libraingun_hip.so abvar/g64/libraingun_hip.so abvar/g256/libraingun_hip.so abvar/dc25/libraingun_hip.so abvar/dc1/libraingun_hip.so"
echo "== north star 50 frames"
bash scripts/ab_bench.sh "--workload synth1024 --no-extra --steps 50 --warmup 5" 2 $L || exit 1
echo "== synth4096p8d8 1920x1080 20 frames"
bash scripts/ab_bench.sh "--workload synth4096p8d8 --width 1920 --height 1080 --no-extra --steps 20 --warmup 3" 1 $L || exit 1
echo session done
