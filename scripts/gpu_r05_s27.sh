#!/bin/bash
# session 27: no tile-slot prefetch in the light path's persistent single launches (TPW < 0) vs HEAD
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s27
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/s27/pytest.log 2>&1
tail -1 gpurun_out/s27/pytest.log
for r in 1 2; do
for v in abvar/head raingun_amd; do
  RAINGUN_HIP_LIB=$PWD/$v/libraingun_hip.so timeout -k 10 300 python scripts/latency_probe.py test1 test3 > gpurun_out/s27/lat_$(basename $v)_$r.json 2> gpurun_out/s27/lat_$(basename $v)_$r.err
  python - gpurun_out/s27/lat_$(basename $v)_$r.json $v <<'PY'
import json, sys
D = json.load(open(sys.argv[1]))
for wl in ("test1", "test3"):
    d = D[wl]
    print(sys.argv[2], wl, "whole", d["whole_kernel_ms"], "share8_max", d["share8_max_ms"], "pinned", d["host_pinned_1gpu_ms"],
          "multi", d["multi_8gpu_rehearsal"]["projected_ms_per_step"], d["multi_8gpu_rehearsal"]["projected_speedup_vs_1gpu"])
PY
done
done
bash scripts/ab_bench.sh "--workload test1 --no-extra --steps 200 --warmup 5" 2 abvar/head/libraingun_hip.so raingun_amd/libraingun_hip.so
