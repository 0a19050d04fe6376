#!/bin/bash
# Round-4 session 11: the driver's own configuration (--steps 20 --warmup 5)
# and a long one (200 steps), interleaved, for the default library and the
# tiles-per-wave / MAXD-4 variants.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for W in test1 test3; do
  for S in 20 200; do
    echo "== $W steps $S"
    bash scripts/ab_bench.sh "--workload $W --no-extra --steps $S --warmup 5" 3 abvar/base/libraingun_hip.so abvar/btpw16/libraingun_hip.so abvar/m4/libraingun_hip.so || exit 1
  done
done
echo "== synth1024 steps 20"
bash scripts/ab_bench.sh "--workload synth1024 --no-extra --steps 20 --warmup 5" 2 abvar/base/libraingun_hip.so abvar/m4/libraingun_hip.so || exit 1
echo session done
