#!/bin/bash
# Round-4: is a single launch throttled by the runtime's scratch limit?  The
# launch-mode probe and the single-launch latency probe, default vs a raised
# per-dispatch scratch limit vs the scratch thread limiter off.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_scratch; mkdir -p $O
timeout -k 10 200 python scripts/launch_probe.py test1 synth1024 > $O/launch_base.json 2> $O/launch_base.err || { tail $O/launch_base.err; exit 1; }
cat $O/launch_base.json
HSA_SCRATCH_SINGLE_LIMIT=8000000000 timeout -k 10 200 python scripts/launch_probe.py test1 synth1024 > $O/launch_lim8g.json 2> $O/launch_lim8g.err || { tail $O/launch_lim8g.err; exit 1; }
cat $O/launch_lim8g.json
HSA_NO_SCRATCH_THREAD_LIMITER=1 timeout -k 10 200 python scripts/launch_probe.py test1 synth1024 > $O/launch_nolim.json 2> $O/launch_nolim.err || { tail $O/launch_nolim.err; exit 1; }
cat $O/launch_nolim.json
HSA_SCRATCH_SINGLE_LIMIT=8000000000 timeout -k 10 240 python scripts/latency_probe.py test1 synth1024 > $O/lat_lim8g.json 2> $O/lat_lim8g.err || { tail $O/lat_lim8g.err; exit 1; }
cat $O/lat_lim8g.json
