#!/bin/bash
# Round-4 session 9: shading frames in global memory (no 704-B scratch array per
# lane, so no slow scratch-wave dispatch): interleaved A/B on bench.py's timed
# configuration (test1, test3, north star) and single-launch latency.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/r04_s9; mkdir -p "$O"
export TMPDIR=/tmp
for W in test1 test3 synth1024; do
  echo "== $W"
  steps=200; [ $W = synth1024 ] && steps=40
  bash scripts/ab_bench.sh "--workload $W --no-extra --steps $steps" 3 abvar/base/libraingun_hip.so abvar/gf/libraingun_hip.so abvar/gfa/libraingun_hip.so || exit 1
done
for v in gfa; do
  RAINGUN_HIP_LIB=$R/abvar/$v/libraingun_hip.so timeout -k 10 240 python scripts/latency_probe.py test1 synth1024 > "$O/lat_$v.json" 2> "$O/lat_$v.err" || { tail "$O/lat_$v.err"; exit 1; }
  echo "$v"; python - "$O/lat_$v.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for w in ("test1", "synth1024"):
    r = d[w]; m = r["multi_8gpu_rehearsal"]
    print(f"  {w}: whole {r['whole_kernel_ms']} share8 max {r['share8_max_ms']} host1 {r['host_pinned_1gpu_ms']} multi {m['projected_ms_per_step']} x{m['projected_speedup_vs_1gpu']}")
PY
done
echo session done
