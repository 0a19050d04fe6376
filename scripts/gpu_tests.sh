#!/bin/bash
# GPU test session: the -m gpu suite (one process), each test under a thread timeout.
# usage: bash scripts/gpu_tests.sh [pytest selection args...]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 180 --timeout-method thread -m gpu "${@:-tests/}" > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -5 gpurun_out/gpu_tests.log
grep -E "FAILED|ERROR|Error" gpurun_out/gpu_tests.log | head -20
exit $rc
