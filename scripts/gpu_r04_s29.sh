#!/bin/bash
# Round-4 session 29: light tiles per wave 12 / 20 (t12 / t20) against HEAD's 16
# (in-tree library) with the tile-slot prefetch in place: test1 at 20 and 200
# frames, test3 at 20, interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for S in 20 200; do
  echo "== test1 steps $S"
  bash scripts/ab_bench.sh "--workload test1 --no-extra --steps $S --warmup 5" 2 raingun_amd/libraingun_hip.so abvar/t12/libraingun_hip.so abvar/t20/libraingun_hip.so || exit 1
done
echo "== test3 steps 20"
bash scripts/ab_bench.sh "--workload test3 --no-extra --steps 20 --warmup 5" 2 raingun_amd/libraingun_hip.so abvar/t12/libraingun_hip.so abvar/t20/libraingun_hip.so || exit 1
echo session done
