#!/bin/bash
# Round-5 session 4: shadow-ray light buffers (rg_lightbuf.cpp).  The whole -m gpu suite on the
# in-tree library, then interleaved A/Bs against the library before them (abvar/base, 10583a3):
# north star 50 frames, the configs[4] scene at 1080p, test1 (light path: unchanged code) 50.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05_s4; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B=abvar/base/libraingun_hip.so; N=raingun_amd/libraingun_hip.so
echo "== north star 50 frames"
bash scripts/ab_bench.sh "--workload synth1024 --no-extra --steps 50 --warmup 5" 3 $B $N || exit 1
echo "== synth4096p8d8 1920x1080 20 frames"
bash scripts/ab_bench.sh "--workload synth4096p8d8 --width 1920 --height 1080 --no-extra --steps 20 --warmup 3" 2 $B $N || exit 1
echo "== test1 50 frames"
bash scripts/ab_bench.sh "--workload test1 --no-extra --steps 50 --warmup 5" 2 $B $N || exit 1
echo session done
