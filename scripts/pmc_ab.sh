#!/bin/bash
# PMC A/B of library variants: one --pmc pass per counter group and library on bench.py's
# timed configuration; per-frame counter values (rocprof sums the counter over one dispatch
# = one frame) are printed by scripts/pmc_ab.py.
#   bash scripts/pmc_ab.sh <workload> "<counters>" lib1 lib2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; W=$1; CNT=$2; shift 2
export TMPDIR=/tmp
for lib in "$@"; do
  tag=$(echo "$lib" | tr '/' '_')
  OUT=$R/gpurun_out/pmcab/$W/$tag
  mkdir -p "$OUT"
  (cd /tmp && RAINGUN_HIP_LIB=$R/$lib timeout -s KILL 240 rocprofv3 --pmc $CNT --kernel-trace --output-format csv -d "$OUT" -o run -- \
      python3 $R/bench.py --workload $W --no-extra --no-cpu-baseline --roofline-frames 1 --steps 3 --warmup 1 > "$OUT/log" 2>&1)
  rc=$?
  echo "$W $lib rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/log"; exit $rc; fi
  python3 scripts/pmc_ab.py "$OUT" "$lib"
done
