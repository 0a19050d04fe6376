#!/bin/bash
# Per-kernel durations of two library variants (rocprofv3 --kernel-trace --stats),
# one bench.py run of a workload each:  bash scripts/ab_kernels.sh <workload> lib1 lib2 ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; W=$1; shift
mkdir -p gpurun_out/abk
export TMPDIR=/tmp
for lib in "$@"; do
  tag=$(echo "$lib" | tr '/' '_')
  (cd /tmp && RAINGUN_HIP_LIB=$R/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$R/gpurun_out/abk/$tag" -o run -- python3 "$R/bench.py" --workload "$W" --no-extra --no-cpu-baseline \
      --steps 100 --warmup 5 > "$R/gpurun_out/abk/$tag.json" 2> "$R/gpurun_out/abk/$tag.err") || { echo "FAIL $lib"; exit 1; }
  echo "== $lib"; cut -d, -f1-5 "$R/gpurun_out/abk/$tag/run_kernel_stats.csv" | head -8
done
