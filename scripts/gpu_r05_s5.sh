#!/bin/bash
# Round-5 session 5: light buffers v2 (list entries four at a time; the camera buffer for primary
# rays).  GPU parity subset, then A/B against v1 (abvar/lb1, 2ad5d10) and the library before the
# buffers (abvar/base): north star 50 frames, the configs[4] scene at 1080p.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05_s5; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B=abvar/base/libraingun_hip.so; L1=abvar/lb1/libraingun_hip.so; N=raingun_amd/libraingun_hip.so
echo "== north star 50 frames"
bash scripts/ab_bench.sh "--workload synth1024 --no-extra --steps 50 --warmup 5" 3 $B $L1 $N || exit 1
echo "== synth4096p8d8 1920x1080 20 frames"
bash scripts/ab_bench.sh "--workload synth4096p8d8 --width 1920 --height 1080 --no-extra --steps 20 --warmup 3" 2 $B $L1 $N || exit 1
echo session done
