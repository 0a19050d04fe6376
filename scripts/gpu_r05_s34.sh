#!/bin/bash
# session 34: light persistent single launches (rg_render_multi shares) at 8 / 12 / 16 one-wave blocks per CU,
# now that they no longer prefetch tile slots
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s34
for r in 1 2; do
for v in raingun_amd abvar/p12 abvar/p16; do
  RAINGUN_HIP_LIB=$PWD/$v/libraingun_hip.so timeout -k 10 300 python scripts/latency_probe.py test1 test3 > gpurun_out/s34/lat_$(basename $v)_$r.json 2> gpurun_out/s34/lat_$(basename $v)_$r.err
  python -c "
import json,sys
D=json.load(open(sys.argv[1]))
for wl in ('test1','test3'):
    d=D[wl]; print(sys.argv[2], wl, 'share8_max', d['share8_max_ms'], 'multi', d['multi_8gpu_rehearsal']['projected_ms_per_step'])" gpurun_out/s34/lat_$(basename $v)_$r.json $v
done
done
