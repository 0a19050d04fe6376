#!/bin/bash
# session 36: RG_LIGHT_PERSIST_BLOCKS_PER_CU 6 at HEAD: full GPU suite, shares
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s36
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/s36/pytest.log 2>&1 || { tail -30 gpurun_out/s36/pytest.log; exit 1; }
tail -1 gpurun_out/s36/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s36/smoke.log 2>&1 || { tail gpurun_out/s36/smoke.log; exit 1; }
tail -1 gpurun_out/s36/smoke.log
timeout -k 10 300 python scripts/latency_probe.py test1 test3 > gpurun_out/s36/lat.json 2> gpurun_out/s36/lat.err
python -c "
import json
D=json.load(open('gpurun_out/s36/lat.json'))
for wl in ('test1','test3'):
    d=D[wl]; print(wl, 'share8_max', d['share8_max_ms'], 'multi', d['multi_8gpu_rehearsal']['projected_ms_per_step'], d['multi_8gpu_rehearsal']['projected_speedup_vs_1gpu'])"
