#!/bin/bash
# scripts/pmc_work.sh for every bench line (BASELINE configs[1..4] + north_star); stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for spec in "test1 3840 2160 20" "test3 3840 2160 20" "synth1024 3840 2160 20" "synth1024 7680 4320 10" "synth4096p8d8 16384 16384 4"; do
  set -- $spec
  bash scripts/pmc_work.sh $1 $2 $3 $4 || exit $?
done
