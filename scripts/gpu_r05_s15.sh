#!/bin/bash
# session 15: host-frame features on the MAXD=8 array-frame kernels (HF) vs the MAXD=0 global-frame kernels (hf0)
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s15
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_paths.py tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/s15/pytest.log 2>&1
tail -1 gpurun_out/s15/pytest.log
for r in 1 2; do
for v in abvar/hf0 raingun_amd; do
  RAINGUN_HIP_LIB=$PWD/$v/libraingun_hip.so timeout -k 10 300 python scripts/hv_sweep.py --workload synth1024 0 -1:4 | sed "s|^|$v |" | tee -a gpurun_out/s15/hv_ns.txt
  RAINGUN_HIP_LIB=$PWD/$v/libraingun_hip.so timeout -k 10 300 python scripts/hv_sweep.py --workload test1 0 | sed "s|^|$v |" | tee -a gpurun_out/s15/hv_t1.txt
done
done
