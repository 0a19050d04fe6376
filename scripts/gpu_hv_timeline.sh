#!/bin/bash
# rocprofv3 timelines of host-visible test1 frames (kernels + memory copies)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; mkdir -p gpurun_out/hvt
export TMPDIR=/tmp
for B in ${HVT_BANDS:-0 8}; do
  (cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/hvt/b$B -o run -- python3 $R/scripts/hv_timeline.py test1 $B) > gpurun_out/hvt/b$B.log 2>&1 || { tail -5 gpurun_out/hvt/b$B.log; exit 1; }
  grep "ms per frame" gpurun_out/hvt/b$B.log
done
