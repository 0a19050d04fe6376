#!/bin/bash
# Memory-instruction mix of one bench workload (dynamic counts per launch):
# VMEM (global + scratch) reads/writes, FLAT, SMEM, LDS -- one --pmc pass.
#   bash scripts/pmc_mem.sh <workload> [width height]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; W=${1:-test1}; X=${2:-3840}; Y=${3:-2160}
OUT=$R/gpurun_out/pmcmem/${W}_${X}x${Y}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_FLAT SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU \
    --kernel-trace --output-format csv -d "$OUT" -o run -- \
    python3 "$R/bench.py" --workload "$W" --width "$X" --height "$Y" --no-extra --no-cpu-baseline --steps 3 --warmup 1 \
    --roofline-frames 1 --settle-s 0 > "$OUT/run.log" 2>&1
