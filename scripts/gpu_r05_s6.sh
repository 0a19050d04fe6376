#!/bin/bash
# Round-5 session 6: where the heavy path's time goes after the light buffers -- BVH walk
# statistics and clocks (abvar/bvhstats, -DRG_BVH_STATS), SIMD use of the query iterations
# (abvar/iterstats, -DRG_ITER_STATS), and the shadow-trace ablation on the current kernel
# (abvar/noshadow2: shadow rays not traced; wrong images, timing only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05_s6; mkdir -p $O
RAINGUN_HIP_LIB=$PWD/abvar/bvhstats/libraingun_hip.so timeout -k 10 300 python scripts/bvh_stats.py > $O/bvh_stats.json 2> $O/bvh_stats.err || { tail $O/bvh_stats.err; exit 1; }
cat $O/bvh_stats.json
RAINGUN_HIP_LIB=$PWD/abvar/iterstats/libraingun_hip.so timeout -k 10 300 python scripts/iter_stats.py synth1024 > $O/iter_stats.json 2> $O/iter_stats.err || { tail $O/iter_stats.err; exit 1; }
cat $O/iter_stats.json
N=raingun_amd/libraingun_hip.so; X=abvar/noshadow2/libraingun_hip.so
echo "== north star 50 frames"
bash scripts/ab_bench.sh "--workload synth1024 --no-extra --steps 50 --warmup 5" 2 $N $X || exit 1
echo session done
