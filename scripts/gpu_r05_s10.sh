#!/bin/bash
# Round-5 session 10: light-buffer list bounds loaded before the plane tests (lbuf_begin / finish)
# (in-tree) against loading them after (abvar/lb3, 9d84d35); GPU parity and host-path tests first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05_s10; mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_host_paths.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
L2=abvar/lb3/libraingun_hip.so; N=raingun_amd/libraingun_hip.so
echo "== north star 50 frames"
bash scripts/ab_bench.sh "--workload synth1024 --no-extra --steps 50 --warmup 5" 3 $L2 $N || exit 1
echo "== synth4096p8d8 1920x1080 20 frames"
bash scripts/ab_bench.sh "--workload synth4096p8d8 --width 1920 --height 1080 --no-extra --steps 20 --warmup 3" 2 $L2 $N || exit 1
echo session done
