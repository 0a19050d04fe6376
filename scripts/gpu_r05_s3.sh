#!/bin/bash
# Round-5 session 3: how much of the heavy path's frame its shadow rays take -- the in-tree
# library against an ablation that skips every shadow query on the heavy path (abvar/noshadow,
# wrong images; timing only), north star and the configs[4] scene at 1080p.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
N=raingun_amd/libraingun_hip.so; X=abvar/noshadow/libraingun_hip.so
echo "== north star 50 frames"
bash scripts/ab_bench.sh "--workload synth1024 --no-extra --steps 50 --warmup 5" 2 $N $X || exit 1
echo "== synth4096p8d8 1920x1080 20 frames"
bash scripts/ab_bench.sh "--workload synth4096p8d8 --width 1920 --height 1080 --no-extra --steps 20 --warmup 3" 2 $N $X || exit 1
echo session done
