#!/bin/bash
# session 33: split host frames as the automatic choice for light scenes into pinned memory; host tests + bench lines
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s33
timeout -k 10 400 python -u -m pytest tests/test_gpu_host_paths.py tests/test_gpu_frames.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/s33/pytest.log 2>&1 || { tail -30 gpurun_out/s33/pytest.log; exit 1; }
tail -1 gpurun_out/s33/pytest.log
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --extra host_visible,host_visible_north_star > gpurun_out/s33/hv.$r.json 2> gpurun_out/s33/hv.$r.err
  python - gpurun_out/s33/hv.$r.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
out = []
for k in ("host_visible", "host_visible_north_star"):
    h = d[k]
    out.append(f"{k}: pinned {h['pinned']['ms_per_step']} pageable {h['pageable']['ms_per_step']} "
               f"multi {h['multi_8gpu_rehearsal']['projected_ms_per_step']} ({h['multi_8gpu_rehearsal']['projected_speedup_vs_1gpu']}x)")
print(" | ".join(out))
PY
done
