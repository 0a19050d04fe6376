#!/bin/bash
# session 30: the N>1 bench path on one GPU: world-1 RCCL rehearsal and gloo ranks on the same device (2 and 4),
# each with the 1-rank frame verification and per-rank times in the line
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_paths.py -x -q -m gpu --timeout 120 --timeout-method thread -k heavy_host_frames > gpurun_out/s30_pytest.log 2>&1 || { tail -30 gpurun_out/s30_pytest.log; exit 1; }
tail -1 gpurun_out/s30_pytest.log
mkdir -p gpurun_out/s30
timeout -k 10 300 python bench.py --rccl-rehearsal --steps 20 --warmup 5 --no-extra --no-cpu-baseline > gpurun_out/s30/rccl_w1.json 2> gpurun_out/s30/rccl_w1.err
tail -c 1500 gpurun_out/s30/rccl_w1.json; echo
for n in 2 4; do
  timeout -k 10 300 python bench.py --gpus $n --backend gloo --same-device --steps 10 --warmup 3 --no-extra --no-cpu-baseline > gpurun_out/s30/gloo_w$n.json 2> gpurun_out/s30/gloo_w$n.err
  tail -c 1500 gpurun_out/s30/gloo_w$n.json; echo
done
for wl in synth1024; do
  timeout -k 10 300 python bench.py --workload $wl --gpus 2 --backend gloo --same-device --steps 6 --warmup 2 --no-extra --no-cpu-baseline > gpurun_out/s30/gloo_w2_$wl.json 2> gpurun_out/s30/gloo_w2_$wl.err
  tail -c 1500 gpurun_out/s30/gloo_w2_$wl.json; echo
done
echo "== compiler flag -amdgpu-use-amdgpu-trackers=1 (abvar/trk) vs HEAD"
L="raingun_amd/libraingun_hip.so abvar/trk/libraingun_hip.so"
bash scripts/ab_bench.sh "--workload test1 --no-extra --steps 200 --warmup 5" 3 $L
bash scripts/ab_bench.sh "--workload synth1024 --no-extra --steps 200 --warmup 5" 3 $L
bash scripts/ab_bench.sh "--workload synth4096p8d8 --width 1920 --height 1080 --no-extra --steps 60 --warmup 3" 2 $L
