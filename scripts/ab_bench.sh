#!/bin/bash
# Interleaved A/B of library variants with bench.py's timed configuration.
#   bash scripts/ab_bench.sh "<bench args>" rounds lib1 lib2 ...   (lib = path to a libraingun_hip.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
ARGS=$1; ROUNDS=$2; shift 2
for r in $(seq 1 $ROUNDS); do
  for lib in "$@"; do
    tag=$(echo "$lib" | tr '/' '_')
    RAINGUN_HIP_LIB=$PWD/$lib timeout -k 10 300 python bench.py $ARGS --no-cpu-baseline > gpurun_out/ab/$tag.$r.json 2> gpurun_out/ab/$tag.$r.err || { echo "FAIL $lib"; tail -5 gpurun_out/ab/$tag.$r.err; exit 1; }
    python - "$lib" gpurun_out/ab/$tag.$r.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
extra = {k: v["ms_per_step"] for k, v in d.items() if isinstance(v, dict) and "ms_per_step" in v}
print(sys.argv[1], "main", d["ms_per_step"], json.dumps(extra))
PY
  done
done
