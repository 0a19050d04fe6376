#!/bin/bash
# session 22: shadow fan-out only in single small launches (TASKS) + RG_PIPE_TILES_PER_WAVE 64, vs 907c057 (abvar/head)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s22
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/s22/pytest.log 2>&1
tail -1 gpurun_out/s22/pytest.log
L="abvar/head/libraingun_hip.so raingun_amd/libraingun_hip.so"
echo "== north star, 200 frames"
bash scripts/ab_bench.sh "--workload synth1024 --no-extra --steps 200 --warmup 5" 3 $L
echo "== synth4096p8d8 1920x1080, 60 frames"
bash scripts/ab_bench.sh "--workload synth4096p8d8 --width 1920 --height 1080 --no-extra --steps 60 --warmup 3" 3 $L
echo "== north star 8K, 40 frames"
bash scripts/ab_bench.sh "--workload synth1024 --width 7680 --height 4320 --no-extra --steps 40 --warmup 3" 2 $L
echo "== synth4096p8d8 16384x16384, 4 frames"
bash scripts/ab_bench.sh "--workload synth4096p8d8 --width 16384 --height 16384 --no-extra --steps 4 --warmup 1" 1 $L
echo "== test1, 200 frames"
bash scripts/ab_bench.sh "--workload test1 --no-extra --steps 200 --warmup 5" 2 $L
echo "== single-launch shares (north star)"
for v in abvar/head raingun_amd; do
  RAINGUN_HIP_LIB=$PWD/$v/libraingun_hip.so timeout -k 10 300 python scripts/latency_probe.py synth1024 > gpurun_out/s22/lat_$(basename $v).json 2> gpurun_out/s22/lat_$(basename $v).err
  python - gpurun_out/s22/lat_$(basename $v).json $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["synth1024"]
print(sys.argv[2], "whole", d["whole_kernel_ms"], "share8_max", d["share8_max_ms"], "pinned", d["host_pinned_1gpu_ms"],
      "multi", d["multi_8gpu_rehearsal"]["projected_ms_per_step"], d["multi_8gpu_rehearsal"]["projected_speedup_vs_1gpu"])
PY
done
