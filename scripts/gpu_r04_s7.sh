#!/bin/bash
# Round-4 session 7: the whole -m gpu suite at HEAD, then single-launch latency of
# the light global-frame variants.   usage: bash scripts/gpu_r04_s7.sh "<variants>" [env for the probes]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/r04_s7; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
for v in $1; do
  env $2 RAINGUN_HIP_LIB=$R/abvar/$v/libraingun_hip.so timeout -k 10 240 python scripts/latency_probe.py test1 synth1024 > "$O/lat_$v.json" 2> "$O/lat_$v.err" || { tail "$O/lat_$v.err"; exit 1; }
  echo "$v"; python - "$O/lat_$v.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for w in ("test1", "synth1024"):
    r = d[w]; m = r["multi_8gpu_rehearsal"]
    print(f"  {w}: whole {r['whole_kernel_ms']} share8 max {r['share8_max_ms']} host1 {r['host_pinned_1gpu_ms']} multi {m['projected_ms_per_step']} x{m['projected_speedup_vs_1gpu']}")
PY
done
echo session done
