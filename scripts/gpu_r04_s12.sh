#!/bin/bash
# Round-4 session 12: light single launches as persistent waves (explicit
# occupancy), with and without expensive-first tile order: single-launch
# latency of the whole test1 frame and its 1/8 shares, host-visible frame,
# rg_render_multi rehearsal; then the driver-configuration A/B (session 11).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/r04_s12; mkdir -p "$O"
export TMPDIR=/tmp
for v in base lp16 lp8 lp16o lp8o hf16 hf12; do
  RAINGUN_HIP_LIB=$R/abvar/$v/libraingun_hip.so timeout -k 10 240 python scripts/latency_probe.py test1 > "$O/lat_$v.json" 2> "$O/lat_$v.err" || { tail "$O/lat_$v.err"; exit 1; }
  echo "$v"; python - "$O/lat_$v.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["test1"]; m = r["multi_8gpu_rehearsal"]
print(f"  test1: whole {r['whole_kernel_ms']} share8 max {r['share8_max_ms']} host1 {r['host_pinned_1gpu_ms']} multi {m['projected_ms_per_step']} x{m['projected_speedup_vs_1gpu']}")
PY
done
[ "$1" = ab ] && bash scripts/gpu_r04_s11.sh
echo session done
