#!/bin/bash
# Round-4 session 26: the heavy path at 2 waves per SIMD (no spills: 183 VGPRs),
# alone (hw2) and with the walk helpers (hw2lh, 207 VGPRs): parity, north star
# A/B against HEAD (in-tree library), single-launch share latency.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_s26; mkdir -p $O
L=$PWD/abvar
for v in hw2 hw2lh; do
  RAINGUN_HIP_LIB=$L/$v/libraingun_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
echo "== synth1024 steps 20"
bash scripts/ab_bench.sh "--workload synth1024 --no-extra --steps 20 --warmup 5" 3 raingun_amd/libraingun_hip.so abvar/hw2/libraingun_hip.so abvar/hw2lh/libraingun_hip.so || exit 1
for v in hw2 hw2lh; do
  RAINGUN_HIP_LIB=$L/$v/libraingun_hip.so timeout -k 10 300 python -u scripts/latency_probe.py synth1024 > $O/latency_$v.json 2> $O/latency_$v.err || { tail -5 $O/latency_$v.err; exit 1; }
  python3 -c "
import json,sys;d=json.load(open(sys.argv[1]));x=d['synth1024'];m=x.get('multi_8gpu_rehearsal') or {}
print(sys.argv[2], 'whole', x['whole_kernel_ms'], 'share8 max', x['share8_max_ms'], 'pinned', x.get('host_pinned_1gpu_ms'), 'multi', m.get('projected_ms_per_step'), m.get('projected_speedup_vs_1gpu'))" $O/latency_$v.json $v
done
echo session done
