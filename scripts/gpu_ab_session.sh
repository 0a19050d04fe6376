#!/bin/bash
# One GPU session: (optional) the -m gpu suite, then interleaved A/B of the
# baseline library (abvar/base) against the in-tree one on three workloads.
#   bash scripts/gpu_ab_session.sh [tests]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "$1" = "tests" ]; then bash scripts/gpu_tests.sh || exit 1; fi
for W in ${AB_WORKLOADS:-test1 test3 synth1024}; do
  echo "== $W"
  bash scripts/ab_bench.sh "--workload $W --no-extra --steps ${AB_STEPS:-200}" ${AB_ROUNDS:-3} abvar/base/libraingun_hip.so raingun_amd/libraingun_hip.so || exit 1
done
