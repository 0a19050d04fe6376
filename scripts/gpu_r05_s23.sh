#!/bin/bash
# session 23: runtime knobs on the heavy lines at HEAD (lane depth, tile order), interleaved; RG_PIPE_MIN_CU_DIV 2/8
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s23
run() {  # label, bench args
  timeout -k 10 200 python bench.py $2 --no-extra --no-cpu-baseline > gpurun_out/s23/r.json 2> gpurun_out/s23/r.err
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'])" gpurun_out/s23/r.json "$1"
}
for r in 1 2 3; do
  for ld in 0 1 2; do
    run "ns ld=$ld" "--workload synth1024 --steps 100 --warmup 5 --lane-depth $ld"
    run "c4 ld=$ld" "--workload synth4096p8d8 --width 1920 --height 1080 --steps 60 --warmup 3 --lane-depth $ld"
  done
  run "ns order=0" "--workload synth1024 --steps 100 --warmup 5 --tile-order 0"
  run "c4 order=0" "--workload synth4096p8d8 --width 1920 --height 1080 --steps 60 --warmup 3 --tile-order 0"
done
echo "== RG_PIPE_MIN_CU_DIV"
L="raingun_amd/libraingun_hip.so abvar/cu2/libraingun_hip.so abvar/cu8/libraingun_hip.so"
bash scripts/ab_bench.sh "--workload synth1024 --no-extra --steps 100 --warmup 5" 2 $L
bash scripts/ab_bench.sh "--workload synth4096p8d8 --width 1920 --height 1080 --no-extra --steps 60 --warmup 3" 2 $L
