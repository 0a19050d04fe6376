#!/bin/bash
# session 14: heavy-path host ring (RG_HOST_RING_HEAVY 0/4/8) x host tile shape, north star into pinned memory
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s14
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_paths.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/s14/pytest.log 2>&1
tail -1 gpurun_out/s14/pytest.log
for r in 1 2; do
for v in abvar/ring0 raingun_amd abvar/ring8; do
  RAINGUN_HIP_LIB=$PWD/$v/libraingun_hip.so timeout -k 10 300 python scripts/hv_sweep.py --workload synth1024 --pinned 0 -1:3 -1:4 -1:5 | sed "s|^|$v |" | tee -a gpurun_out/s14/hv_ns.txt
done
done
for v in abvar/ring0 raingun_amd; do
  RAINGUN_HIP_LIB=$PWD/$v/libraingun_hip.so timeout -k 10 300 python scripts/hv_sweep.py --workload test1 --pinned 0 | sed "s|^|$v |" | tee -a gpurun_out/s14/hv_t1.txt
done
