#!/bin/bash
# Round-4 session 15: light path with the texel load issued at the hit (te) on
# test1 / test3; heavy path with the per-lane walk's stack top in a register
# (ltop) on the north star -- interleaved, 20 and 200 frames.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for W in test1 test3; do
  for S in 20 200; do
    echo "== $W steps $S"
    bash scripts/ab_bench.sh "--workload $W --no-extra --steps $S --warmup 5" 3 abvar/base/libraingun_hip.so abvar/te/libraingun_hip.so || exit 1
  done
done
for S in 20 60; do
  echo "== synth1024 steps $S"
  bash scripts/ab_bench.sh "--workload synth1024 --no-extra --steps $S --warmup 5" 3 abvar/base/libraingun_hip.so abvar/ltop/libraingun_hip.so || exit 1
done
echo session done
