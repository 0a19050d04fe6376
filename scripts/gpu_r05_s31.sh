#!/bin/bash
# session 31: split host-visible frames (image bands -2: top pct% rows device-resident + DMA beside a one-launch rest)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s31
timeout -k 10 400 python -u -m pytest tests/test_gpu_host_paths.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/s31/pytest.log 2>&1 || { tail -30 gpurun_out/s31/pytest.log; exit 1; }
tail -1 gpurun_out/s31/pytest.log
for wl in test1 test3 synth1024; do
  timeout -k 10 300 python scripts/hv_sweep.py --workload $wl --pinned -1 -2:0:-1:25 -2:0:-1:35 -2:0:-1:45 -2:0:-1:55 -2:0:-1:65 -1 -2:0:-1:45 | tee -a gpurun_out/s31/hv.jsonl
done
