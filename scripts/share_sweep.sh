#!/bin/bash
# bench.py --share diagnostics: ms per frame of one rank's 1/S share, several settings.
#   bash scripts/share_sweep.sh   (edit the loops for the sweep at hand)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
run() {
  GPU_MAX_HW_QUEUES=16 timeout -k 10 120 python bench.py --no-extra --no-cpu-baseline "$@" > gpurun_out/s.json 2>/dev/null || exit 1
  python -c "import json,sys;d=json.loads(open('gpurun_out/s.json').read().strip().splitlines()[-1]);print(' '.join(sys.argv[1:]), d['ms_per_step'])" "$@"
}
for i in 1 2; do
  run --workload test1 --steps 20 --warmup 5 --frames-in-flight 8
  run --workload test1 --steps 20 --warmup 500 --frames-in-flight 8
  run --workload test1 --steps 200 --warmup 5 --frames-in-flight 8
  run --workload test1 --steps 2000 --warmup 5 --frames-in-flight 8
done
