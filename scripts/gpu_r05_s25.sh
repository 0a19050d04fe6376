#!/bin/bash
# session 25: light-buffer cell records with the list's first two entries inline vs HEAD (abvar/head)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s25
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/s25/pytest.log 2>&1
tail -1 gpurun_out/s25/pytest.log
L="abvar/head/libraingun_hip.so raingun_amd/libraingun_hip.so"
echo "== north star, 200 frames"
bash scripts/ab_bench.sh "--workload synth1024 --no-extra --steps 200 --warmup 5" 3 $L
echo "== synth4096p8d8 1920x1080, 60 frames"
bash scripts/ab_bench.sh "--workload synth4096p8d8 --width 1920 --height 1080 --no-extra --steps 60 --warmup 3" 3 $L
echo "== north star 8K, 40 frames"
bash scripts/ab_bench.sh "--workload synth1024 --width 7680 --height 4320 --no-extra --steps 40 --warmup 3" 2 $L
