#!/bin/bash
# Round-4 session 20: per-lane walk with helpers, variants (own result in the
# slot: lh2; balancing below 24 / 52 walking lanes; 3 matching rounds per
# step), north star A/B against HEAD, parity of the chosen variants, and the
# single-launch share latency + rg_render_multi rehearsal of the north star.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_s20; mkdir -p $O
L=$PWD/abvar
for v in lh2 lh2r3; do
  RAINGUN_HIP_LIB=$L/$v/libraingun_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
echo "== synth1024 steps 20"
bash scripts/ab_bench.sh "--workload synth1024 --no-extra --steps 20 --warmup 5" 2 abvar/base/libraingun_hip.so abvar/lh2/libraingun_hip.so abvar/lh2a24/libraingun_hip.so abvar/lh2a52/libraingun_hip.so abvar/lh2r3/libraingun_hip.so || exit 1
for v in base lh2 lh2r3; do
  RAINGUN_HIP_LIB=$L/$v/libraingun_hip.so timeout -k 10 300 python -u scripts/latency_probe.py synth1024 > $O/latency_$v.json 2> $O/latency_$v.err || { tail -5 $O/latency_$v.err; exit 1; }
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], json.dumps(d)[:600])" $O/latency_$v.json
done
echo session done
