#!/bin/bash
# Kernel trace of bench.py at a rank's 1/S share (frames in flight), to see the
# per-frame GPU-busy union and the small kernels around each render.
#   bash scripts/share_trace.sh <workload> <S> [steps]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; W=${1:-synth1024}; S=${2:-8}; STEPS=${3:-200}
OUT=$R/gpurun_out/share_trace/${W}_s$S
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
    python3 "$R/bench.py" --workload "$W" --share "$S" --no-extra --no-cpu-baseline --steps "$STEPS" --warmup 5 \
    --roofline-frames 1 > "$OUT/bench.json" 2> "$OUT/bench.err"
