#!/bin/bash
# Which engine carries device-to-host copies into page-locked memory (blit kernels vs
# SDMA) under a few runtime settings, and at what rate (scripts/d2h_engine_probe.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; mkdir -p gpurun_out/d2h; export TMPDIR=/tmp
env | grep -iE "sdma|hsa_|^hip|^gpu_|^roc" > gpurun_out/d2h/env.txt
i=0
for E in "X=1" "HSA_ENABLE_SDMA=1" "GPU_FORCE_BLIT_COPY_SIZE=0" "HSA_ENABLE_SDMA=1 GPU_FORCE_BLIT_COPY_SIZE=0"; do
  i=$((i+1))
  echo "== $E"
  (export $E; cd /tmp && timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $R/gpurun_out/d2h/t$i -o run -- python3 $R/scripts/d2h_engine_probe.py) > gpurun_out/d2h/t$i.log 2>&1 || { tail -3 gpurun_out/d2h/t$i.log; exit 1; }
  grep -A20 "^{" gpurun_out/d2h/t$i.log | tr -d '\n ' ; echo
  cut -c1-100 gpurun_out/d2h/t$i/run_kernel_stats.csv | grep -i copy || true
  ls gpurun_out/d2h/t$i/ | tr '\n' ' '; echo
  [ -f gpurun_out/d2h/t$i/run_memory_copy_stats.csv ] && cut -c1-120 gpurun_out/d2h/t$i/run_memory_copy_stats.csv
done
exit 0
