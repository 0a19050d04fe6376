#!/bin/bash
# host-visible test1 (pinned) ms per frame by band count (scripts/hv_timeline.py)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for B in 0 -1 2 3 4 6 8 12 16; do timeout -k 10 120 python scripts/hv_timeline.py ${HVB_WL:-test1} $B 2>&1 | grep "ms per" || exit 1; done
