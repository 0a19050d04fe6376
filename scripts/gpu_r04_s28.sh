#!/bin/bash
# Round-4 session 28: rg_render_multi's 8-device rehearsal per band count
# (HEAD, in-tree library), with a whole-frame equality check per setting.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_s28; mkdir -p $O
timeout -k 10 600 python -u scripts/multi_bands_sweep.py test1 test3 synth1024 > $O/bands.jsonl 2> $O/bands.err || { tail -5 $O/bands.err; exit 1; }
python3 -c "
import json
for l in open('$O/bands.jsonl'):
    d=json.loads(l); print(d['workload'], d['bands'], d['projected_ms'], d['frame_equal'])"
echo session done
