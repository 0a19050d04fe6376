#!/bin/bash
# session 17: north-star breakdown at HEAD: BVH statistics, iteration statistics, time by recursion depth
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s17
RAINGUN_HIP_LIB=$PWD/abvar/bvhstats/libraingun_hip.so timeout -k 10 200 python scripts/bvh_stats.py > gpurun_out/s17/bvh_stats.json 2> gpurun_out/s17/bvh_stats.err
RAINGUN_HIP_LIB=$PWD/abvar/iterstats/libraingun_hip.so timeout -k 10 200 python scripts/iter_stats.py synth1024 test1 > gpurun_out/s17/iter_stats.txt 2> gpurun_out/s17/iter_stats.err
for d in 1 2 3 5; do
  timeout -k 10 200 python bench.py --workload synth1024 --depth $d --steps 100 --warmup 5 --no-extra --no-cpu-baseline > gpurun_out/s17/ns_d$d.json 2> gpurun_out/s17/ns_d$d.err
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print('depth', sys.argv[2], d['ms_per_step'], d.get('rays_per_frame'), d.get('kernel_ms'))" gpurun_out/s17/ns_d$d.json $d
done
cat gpurun_out/s17/bvh_stats.json gpurun_out/s17/iter_stats.txt
