#!/bin/bash
# Executed-work profile of one bench line AT ITS TIMED CONFIGURATION (the bench's
# frames in flight): a kernel-trace --stats pass (per-launch durations; their per-frame
# union is compared with bench.py's ms_per_step by scripts/pmc_work.py) and
# --pmc passes (instruction mix, HBM bytes).  Each pass is its own run, counters
# within one block's limits, nothing but --kernel-trace beside --pmc.
#   bash scripts/pmc_work.sh <workload> <width> <height> [steps]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; W=${1:-test1}; X=${2:-3840}; Y=${3:-2160}; STEPS=${4:-10}
TAG=${W}_${X}x${Y}
OUT=$R/gpurun_out/pmcw/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
BENCH="$R/bench.py --workload $W --width $X --height $Y --no-extra --no-cpu-baseline --roofline-frames 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
    python3 $BENCH --steps $STEPS --warmup 2 > "$OUT/trace.json" 2> "$OUT/trace.err"
rc=$?; echo "$TAG trace rc=$rc"
if [ $rc -ne 0 ]; then tail -5 "$OUT/trace.err"; exit $rc; fi
i=0
for pass in "SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_TRANS_F32 SQ_WAVES SQ_BUSY_CYCLES" \
            "FETCH_SIZE" "WRITE_SIZE" \
            "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_INT64"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d "$OUT/p$i" -o run -- \
      python3 $BENCH --steps 3 --warmup 1 > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "$TAG pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/p$i.log"; exit $rc; fi
done
