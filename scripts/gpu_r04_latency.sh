#!/bin/bash
# Round-4 single-launch latency session: GPU tests of the touched host paths, then
# latency_probe.py (whole frame and every 1/8 share as ONE launch, host-visible
# frame, 8-device rg_render_multi rehearsal) for the default library and the
# variants under abvar/, tile timelines (RG_TILE_TIMES builds), and a kernel
# trace of the single-launch probe.   usage: bash scripts/gpu_r04_latency.sh [variant ...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/r04_latency; mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_frames.py \
    tests/test_gpu_host_paths.py > "$O/pytest.log" 2>&1 || { tail -20 "$O/pytest.log"; exit 1; }
tail -2 "$O/pytest.log"
timeout -k 10 240 python scripts/latency_probe.py test1 synth1024 > "$O/base.json" 2> "$O/base.err" || { tail "$O/base.err"; exit 1; }
echo base; cat "$O/base.json"
timeout -k 10 240 python scripts/latency_probe.py --tile-order test1 > "$O/base_order.json" 2> "$O/base_order.err" || { tail "$O/base_order.err"; exit 1; }
echo base_order; cat "$O/base_order.json"
for v in "$@"; do
  case $v in
    tt*) RAINGUN_HIP_LIB=$R/abvar/$v/libraingun_hip.so timeout -k 10 240 python scripts/tail_probe.py timeline > "$O/$v.json" 2> "$O/$v.err" || { tail "$O/$v.err"; exit 1; } ;;
    *) RAINGUN_HIP_LIB=$R/abvar/$v/libraingun_hip.so timeout -k 10 240 python scripts/latency_probe.py test1 synth1024 > "$O/$v.json" 2> "$O/$v.err" || { tail "$O/$v.err"; exit 1; } ;;
  esac
  echo "$v"; cat "$O/$v.json"
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- \
    python3 "$R/scripts/latency_probe.py" --no-multi test1 synth1024 > "$O/trace_probe.json" 2> "$O/trace_probe.err" || { tail "$O/trace_probe.err"; exit 1; }
echo trace done
