#!/bin/bash
# Round-5 session 11: BVH nodes in LDS when the sphere tables do not fit (in-tree) against global
# nodes (abvar/lb4, HEAD before it): parity incl. the configs[4]-shape and full-size tests, then
# the configs[4] scene at 1080p and at its full 16384^2, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05_s11; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
P=abvar/lb4/libraingun_hip.so; N=raingun_amd/libraingun_hip.so
echo "== synth4096p8d8 1920x1080 20 frames"
bash scripts/ab_bench.sh "--workload synth4096p8d8 --width 1920 --height 1080 --no-extra --steps 20 --warmup 3" 3 $P $N || exit 1
echo "== synth4096p8d8 16384x16384 5 frames"
bash scripts/ab_bench.sh "--workload synth4096p8d8 --width 16384 --height 16384 --no-extra --steps 5 --warmup 2 --roofline-frames 1" 1 $P $N || exit 1
echo session done
