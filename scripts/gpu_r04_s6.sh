#!/bin/bash
# Round-4: fixed per-launch cost of scratch-using kernels (scratch_probe), with
# and without the runtime's scratch reclaim; then the launch-mode probe with
# reclaim off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_s6; mkdir -p $O
timeout -k 10 60 scripts/bin/scratch_probe > $O/scratch_default.txt && cat $O/scratch_default.txt || exit 1
HSA_NO_SCRATCH_RECLAIM=1 timeout -k 10 60 scripts/bin/scratch_probe > $O/scratch_noreclaim.txt && cat $O/scratch_noreclaim.txt || exit 1
HSA_NO_SCRATCH_RECLAIM=1 timeout -k 10 200 python scripts/launch_probe.py test1 synth1024 > $O/launch_noreclaim.json 2> $O/launch_noreclaim.err || { tail $O/launch_noreclaim.err; exit 1; }
cat $O/launch_noreclaim.json
