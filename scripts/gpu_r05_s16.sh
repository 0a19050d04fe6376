#!/bin/bash
# session 16: heavy host frames on array-frame kernels + 16x4 host tiles vs HEAD (907c057), bench host_visible lines
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s16
timeout -k 10 400 python -u -m pytest tests/test_gpu_host_paths.py tests/test_gpu_parity.py tests/test_gpu_frames.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/s16/pytest.log 2>&1
tail -1 gpurun_out/s16/pytest.log
for r in 1 2; do
for v in abvar/head raingun_amd; do
  RAINGUN_HIP_LIB=$PWD/$v/libraingun_hip.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --extra host_visible,host_visible_north_star > gpurun_out/s16/$(basename $v).$r.json 2> gpurun_out/s16/$(basename $v).$r.err
  python - gpurun_out/s16/$(basename $v).$r.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
out = [sys.argv[2]]
for k in ("host_visible", "host_visible_north_star"):
    h = d[k]
    out.append(f"{k}: pinned {h['pinned']['ms_per_step']} pageable {h['pageable']['ms_per_step']} "
               f"multi {h['multi_8gpu_rehearsal']['projected_ms_per_step']} ({h['multi_8gpu_rehearsal']['projected_speedup_vs_1gpu']}x)")
print(" | ".join(out))
PY
done
done
