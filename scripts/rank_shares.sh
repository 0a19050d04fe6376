#!/bin/bash
# Per-rank 1/8 shares on one GPU (bench.py --share 8 --share-rank r, 8 frames in flight) next to the
# whole frame: the bound on 8-GPU scaling before the gather.
#   usage: bash scripts/rank_shares.sh [workload[/WxH] ...]   (e.g. synth1024/7680x4320)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/shares
for spec in "${@:-test1 synth1024}"; do
  wl=${spec%%/*}; size=""; tag=$wl
  if [ "$spec" != "$wl" ]; then sz=${spec#*/}; size="--width ${sz%x*} --height ${sz#*x}"; tag=${wl}_$sz; fi
  steps=200; [ "$wl" = "test1" ] || steps=40; [ -z "$size" ] || steps=20
  for r in whole 0 1 2 3 4 5 6 7; do
    if [ "$r" = whole ]; then extra=""; else extra="--share 8 --share-rank $r"; fi
    timeout -k 10 180 python bench.py --workload $wl $size --no-extra --no-cpu-baseline --steps $steps $extra > gpurun_out/shares/$tag.$r.json 2>gpurun_out/shares/$tag.$r.err || { echo "FAIL $wl $r"; tail -3 gpurun_out/shares/$tag.$r.err; exit 1; }
    python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);print(sys.argv[2], sys.argv[3], d['ms_per_step'])" gpurun_out/shares/$tag.$r.json $tag $r
  done
done
