#!/bin/bash
# Round-4 combined diagnostics (one box): GPU suite at HEAD; scratch-using
# dispatch cost with and without the runtime's scratch reclaim; launch-mode
# probe with reclaim off; single-launch latency of the light global-frame
# variants; tile timelines of 1/8 shares (4 tiles per wave; BVH stats).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/r04_s8; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 60 scripts/bin/scratch_probe > $O/scratch_default.txt && cat $O/scratch_default.txt || exit 1
HSA_NO_SCRATCH_RECLAIM=1 timeout -k 10 60 scripts/bin/scratch_probe > $O/scratch_noreclaim.txt && cat $O/scratch_noreclaim.txt || exit 1
HSA_NO_SCRATCH_RECLAIM=1 timeout -k 10 200 python scripts/launch_probe.py test1 > $O/launch_noreclaim.json 2> $O/launch_noreclaim.err || { tail $O/launch_noreclaim.err; exit 1; }
cat $O/launch_noreclaim.json; echo
# one call's tiles split over k launches on k streams (hardware queues), 4 tiles per wave
GPU_MAX_HW_QUEUES=8 RAINGUN_HIP_LIB=$R/abvar/gft4/libraingun_hip.so timeout -k 10 200 python scripts/launch_probe.py test1 > $O/launch_gft4_q8.json 2> $O/launch_gft4_q8.err || { tail $O/launch_gft4_q8.err; exit 1; }
cat $O/launch_gft4_q8.json; echo
for v in gf gfsp gft4; do
  RAINGUN_HIP_LIB=$R/abvar/$v/libraingun_hip.so timeout -k 10 240 python scripts/latency_probe.py test1 > "$O/lat_$v.json" 2> "$O/lat_$v.err" || { tail "$O/lat_$v.err"; exit 1; }
  echo "$v"; python - "$O/lat_$v.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
r = d["test1"]; m = r["multi_8gpu_rehearsal"]
print(f"  test1: whole {r['whole_kernel_ms']} share8 max {r['share8_max_ms']} host1 {r['host_pinned_1gpu_ms']} multi {m['projected_ms_per_step']} x{m['projected_speedup_vs_1gpu']}")
PY
done
for v in tttpw4 ttbs; do
  RAINGUN_HIP_LIB=$R/abvar/$v/libraingun_hip.so timeout -k 10 240 python scripts/tail_probe.py timeline > "$O/tl_$v.json" 2> "$O/tl_$v.err" || { tail "$O/tl_$v.err"; exit 1; }
done
echo session done
