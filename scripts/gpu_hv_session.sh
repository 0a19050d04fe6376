#!/bin/bash
# GPU session: the -m gpu suite, then the host-visible lines (rg_render_image pinned /
# pageable, and the rg_render_multi 8-GPU timeline rehearsal) for test1 and the north star.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "$1" != "notests" ]; then bash scripts/gpu_tests.sh || exit 1; fi
timeout -k 10 400 python bench.py --extra host_visible,host_visible_north_star --no-cpu-baseline --steps 50 \
    > gpurun_out/bench_hv.json 2> gpurun_out/bench_hv.err || { tail -20 gpurun_out/bench_hv.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/bench_hv.json").read().strip().splitlines()[-1])
print("main", d["ms_per_step"], d["value"])
for k in ("host_visible", "host_visible_north_star"):
    v = d[k]
    print(k, "pinned", v["pinned"]["ms_per_step"], "pageable", v["pageable"]["ms_per_step"])
    print("  ", json.dumps(v["multi_8gpu_rehearsal"]))
PY
