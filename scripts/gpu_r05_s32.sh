#!/bin/bash
# session 32: split host-visible frames, finer fraction sweep; part B launched first (abvar/bfirst)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s32
for r in 1 2; do
for v in raingun_amd abvar/bfirst; do
for wl in test1 test3; do
  RAINGUN_HIP_LIB=$PWD/$v/libraingun_hip.so timeout -k 10 300 python scripts/hv_sweep.py --workload $wl --pinned -1 -2:0:-1:30 -2:0:-1:35 -2:0:-1:40 -1 -2:0:-1:35 | sed "s|^|$v |" | tee -a gpurun_out/s32/hv.txt
done
done
done
