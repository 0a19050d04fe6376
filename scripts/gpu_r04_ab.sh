#!/bin/bash
# Interleaved A/B of abvar/<variant> libraries against abvar/base on bench.py's
# timed configuration.  usage: bash scripts/gpu_r04_ab.sh "<workloads>" rounds variant ...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
WLS=$1; ROUNDS=$2; shift 2
libs="abvar/base/libraingun_hip.so"
for v in "$@"; do libs="$libs abvar/$v/libraingun_hip.so"; done
for W in $WLS; do
  echo "== $W"
  bash scripts/ab_bench.sh "--workload $W --no-extra --steps 200" "$ROUNDS" $libs || exit 1
done
