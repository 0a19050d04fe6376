#!/bin/bash
# session 20: heavy-path knobs after the light buffers: shadow fan-out, pipelined tiles per wave, per-lane walk depth
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s20
echo "== north star, 100 frames"
bash scripts/ab_bench.sh "--workload synth1024 --no-extra --steps 100 --warmup 5" 2 raingun_amd/libraingun_hip.so abvar/fan0/libraingun_hip.so abvar/fan1/libraingun_hip.so abvar/ptw16/libraingun_hip.so abvar/ptw64/libraingun_hip.so
echo "== synth4096p8d8 1920x1080, 40 frames"
bash scripts/ab_bench.sh "--workload synth4096p8d8 --width 1920 --height 1080 --no-extra --steps 40 --warmup 3" 1 raingun_amd/libraingun_hip.so abvar/fan0/libraingun_hip.so abvar/fan1/libraingun_hip.so abvar/ptw16/libraingun_hip.so abvar/ptw64/libraingun_hip.so
echo "== lane depth, north star / synth4096p8d8 1080p"
for ld in 0 1 2 99; do
  for w in "synth1024" "synth4096p8d8 --width 1920 --height 1080"; do
    timeout -k 10 200 python bench.py --workload $w --lane-depth $ld --steps 60 --warmup 5 --no-extra --no-cpu-baseline > gpurun_out/s20/ld.json 2> gpurun_out/s20/ld.err
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('lane_depth', sys.argv[2], sys.argv[3], d['ms_per_step'])" gpurun_out/s20/ld.json $ld "$w"
  done
done
