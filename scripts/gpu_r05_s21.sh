#!/bin/bash
# session 21: shadow fan-out off (RG_SHADOW_FAN=0) and pipelined tiles per wave 64/128 on the heavy lines; single-launch shares
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s21
RAINGUN_HIP_LIB=$PWD/abvar/f0p64/libraingun_hip.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/s21/pytest.log 2>&1
tail -1 gpurun_out/s21/pytest.log
L="raingun_amd/libraingun_hip.so abvar/fan0/libraingun_hip.so abvar/f0p64/libraingun_hip.so abvar/f0p128/libraingun_hip.so abvar/ptw128/libraingun_hip.so"
echo "== north star, 200 frames"
bash scripts/ab_bench.sh "--workload synth1024 --no-extra --steps 200 --warmup 5" 2 $L
echo "== synth4096p8d8 1920x1080, 60 frames"
bash scripts/ab_bench.sh "--workload synth4096p8d8 --width 1920 --height 1080 --no-extra --steps 60 --warmup 3" 3 $L
echo "== north star 8K, 40 frames"
bash scripts/ab_bench.sh "--workload synth1024 --width 7680 --height 4320 --no-extra --steps 40 --warmup 3" 1 $L
echo "== single-launch shares (north star)"
for v in raingun_amd abvar/fan0 abvar/f0p64; do
  RAINGUN_HIP_LIB=$PWD/$v/libraingun_hip.so timeout -k 10 300 python scripts/latency_probe.py synth1024 > gpurun_out/s21/lat_$(basename $v).json 2> gpurun_out/s21/lat_$(basename $v).err
  python - gpurun_out/s21/lat_$(basename $v).json $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[2], json.dumps(d)[:600])
PY
done
