#!/bin/bash
# session 13: host-visible north star (one launch into pinned memory): tile order / tile shape
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s13
timeout -k 10 300 python scripts/hv_sweep.py --workload synth1024 --pinned 0 -1:3:1 -1:3:0 -1:4:1 -1:4:0 -1:6:0 -1:6:1 3 0 > gpurun_out/s13/hv_ns.jsonl 2> gpurun_out/s13/hv_ns.err
timeout -k 10 300 python scripts/hv_sweep.py --workload test1 --pinned 0 -1:6:0 -1:6:1 -1:3:0 3 0 > gpurun_out/s13/hv_t1.jsonl 2> gpurun_out/s13/hv_t1.err
cat gpurun_out/s13/*.jsonl
