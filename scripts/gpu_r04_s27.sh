#!/bin/bash
# Round-4 session 27: persistent light waves for single launches below the
# whole-frame size (rg_render_multi's shares and bands) at 2 / 3 waves per SIMD
# (sp8 / sp12): the whole -m gpu suite on sp8, then single-launch latency and
# the multi rehearsal against HEAD (in-tree library).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_s27; mkdir -p $O
L=$PWD/abvar
RAINGUN_HIP_LIB=$L/sp8/libraingun_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest_sp8.log 2>&1 || { tail -30 $O/pytest_sp8.log; exit 1; }
tail -1 $O/pytest_sp8.log
for r in 1 2; do
for v in base sp8 sp12; do
  lib=$L/$v/libraingun_hip.so; [ $v = base ] && lib=$PWD/raingun_amd/libraingun_hip.so
  RAINGUN_HIP_LIB=$lib timeout -k 10 300 python -u scripts/latency_probe.py test1 test3 > $O/latency_${v}_$r.json 2> $O/latency_$v.err || { tail -5 $O/latency_$v.err; exit 1; }
  python3 -c "
import json,sys;d=json.load(open(sys.argv[1]))
for w in ('test1','test3'):
    x=d[w]; m=x.get('multi_8gpu_rehearsal') or {}
    print(sys.argv[2], w, 'whole', x['whole_kernel_ms'], 'share8 max', x['share8_max_ms'], 'pinned', x.get('host_pinned_1gpu_ms'), 'multi', m.get('projected_ms_per_step'), m.get('projected_speedup_vs_1gpu'))" $O/latency_${v}_$r.json $v
done
done
echo session done
