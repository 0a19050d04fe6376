#!/bin/bash
# Round-4 session 18: per-lane walk with helpers (RG_LANE_HELP, abvar/lh).
# Walk statistics first (per-lane walk clock share; lanes per walk iteration
# without / with helpers), then parity with the helper build, then an
# interleaved north-star A/B against HEAD.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_s18; mkdir -p $O
L=$PWD/abvar
RAINGUN_HIP_LIB=$L/bs/libraingun_hip.so timeout -k 10 180 python -u scripts/bvh_stats.py > $O/bvh_stats_lane_clock.json 2> $O/bvh_stats.err || { tail -5 $O/bvh_stats.err; exit 1; }
cat $O/bvh_stats_lane_clock.json
RAINGUN_HIP_LIB=$L/it/libraingun_hip.so timeout -k 10 120 python -u scripts/iter_stats.py synth1024 > $O/iter_base.json 2> $O/iter_base.err || { tail -5 $O/iter_base.err; exit 1; }
RAINGUN_HIP_LIB=$L/lhi/libraingun_hip.so timeout -k 10 120 python -u scripts/iter_stats.py synth1024 > $O/iter_lh.json 2> $O/iter_lh.err || { tail -5 $O/iter_lh.err; exit 1; }
cat $O/iter_base.json $O/iter_lh.json
RAINGUN_HIP_LIB=$L/lh/libraingun_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/pytest_lh.log 2>&1 || { tail -30 $O/pytest_lh.log; exit 1; }
tail -1 $O/pytest_lh.log
echo "== synth1024 steps 20"
bash scripts/ab_bench.sh "--workload synth1024 --no-extra --steps 20 --warmup 5" 3 abvar/base/libraingun_hip.so abvar/lh/libraingun_hip.so || exit 1
echo session done
