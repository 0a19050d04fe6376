#!/bin/bash
# Round-4 session 23: light-path tile cap above the wave's share (lc2 / lc4:
# RG_LIGHT_CAP_MUL) -- the whole -m gpu suite on lc4, single-launch latency of
# the whole frame and of the 1/8 shares (+ the multi rehearsal), and the
# pipelined A/B against HEAD (in-tree library).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_s23; mkdir -p $O
L=$PWD/abvar
RAINGUN_HIP_LIB=$L/lc4/libraingun_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest_lc4.log 2>&1 || { tail -30 $O/pytest_lc4.log; exit 1; }
tail -1 $O/pytest_lc4.log
for v in base lc2 lc4; do
  lib=$L/$v/libraingun_hip.so; [ $v = base ] && lib=$PWD/raingun_amd/libraingun_hip.so
  RAINGUN_HIP_LIB=$lib timeout -k 10 300 python -u scripts/latency_probe.py test1 test3 > $O/latency_$v.json 2> $O/latency_$v.err || { tail -5 $O/latency_$v.err; exit 1; }
  python3 -c "
import json,sys;d=json.load(open(sys.argv[1]))
for w in ('test1','test3'):
    x=d[w]; m=x.get('multi_8gpu_rehearsal') or {}
    print(sys.argv[2], w, 'whole', x['whole_kernel_ms'], 'share8 max', x['share8_max_ms'], 'pinned', x.get('host_pinned_1gpu_ms'), 'multi', m.get('projected_ms_per_step'), m.get('projected_speedup_vs_1gpu'))" $O/latency_$v.json $v
done
for S in 20 200; do
  echo "== test1 steps $S"
  bash scripts/ab_bench.sh "--workload test1 --no-extra --steps $S --warmup 5" 2 raingun_amd/libraingun_hip.so abvar/lc2/libraingun_hip.so abvar/lc4/libraingun_hip.so || exit 1
done
echo "== test3 steps 20"
bash scripts/ab_bench.sh "--workload test3 --no-extra --steps 20 --warmup 5" 2 raingun_amd/libraingun_hip.so abvar/lc2/libraingun_hip.so abvar/lc4/libraingun_hip.so || exit 1
echo session done
