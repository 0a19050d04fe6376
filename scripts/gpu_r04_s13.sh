#!/bin/bash
# Round-4 session 13: big light launches at 16 / 24 / 32 tiles per wave in the
# driver's configuration (20 steps, 5 warm-up) and at 200 steps; the pageable
# host-visible frame with 3 vs 7 helper copy threads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for W in test1 test3; do
  for S in 20 200; do
    echo "== $W steps $S"
    bash scripts/ab_bench.sh "--workload $W --no-extra --steps $S --warmup 5" 3 abvar/base/libraingun_hip.so abvar/btpw16/libraingun_hip.so abvar/btpw24/libraingun_hip.so || exit 1
  done
done
echo "== host_visible (test1; pinned, pageable)"
bash scripts/ab_bench.sh "--workload test1 --extra host_visible --steps 40 --warmup 5" 2 abvar/base/libraingun_hip.so abvar/ch7/libraingun_hip.so || exit 1
for f in gpurun_out/ab/abvar_*_libraingun_hip.so.*.json; do
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);h=d.get('host_visible');print(sys.argv[1], h and (h['pinned']['ms_per_step'], h['pageable']['ms_per_step']))" $f
done
echo session done
