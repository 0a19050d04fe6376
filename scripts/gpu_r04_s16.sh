#!/bin/bash
# Round-4 session 16: the -m gpu suite at HEAD (early texel load), then the
# pageable host-visible frame with non-temporal host band copies (cnt) vs HEAD.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_s16; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash scripts/ab_bench.sh "--workload test1 --extra host_visible,host_visible_north_star --steps 40 --warmup 5" 3 abvar/base/libraingun_hip.so abvar/cnt/libraingun_hip.so > $O/ab.txt || exit 1
for f in gpurun_out/ab/abvar_*_libraingun_hip.so.*.json; do
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);h=d['host_visible'];n=d['host_visible_north_star'];print(sys.argv[1].split('/')[-1], 'test1', h['pinned']['ms_per_step'], h['pageable']['ms_per_step'], 'north star', n['pinned']['ms_per_step'], n['pageable']['ms_per_step'])" $f
done
echo session done
