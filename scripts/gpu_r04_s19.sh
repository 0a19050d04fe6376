#!/bin/bash
# Round-4 session 19 (sessions 17 and 18 in one call): the -m gpu suite at HEAD;
# the per-lane walk with helpers (RG_LANE_HELP: walk statistics, parity, north
# star A/B); unwind preload (up) / tile-slot prefetch (tp) vs HEAD on the light
# scenes; pageable host-visible frames with non-temporal host copies (cnt).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_s19; mkdir -p $O
L=$PWD/abvar
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
RAINGUN_HIP_LIB=$L/bs/libraingun_hip.so timeout -k 10 180 python -u scripts/bvh_stats.py > $O/bvh_stats_lane_clock.json 2> $O/bvh_stats.err || { tail -5 $O/bvh_stats.err; exit 1; }
cat $O/bvh_stats_lane_clock.json
RAINGUN_HIP_LIB=$L/it/libraingun_hip.so timeout -k 10 120 python -u scripts/iter_stats.py synth1024 > $O/iter_base.json 2> $O/iter_base.err || { tail -5 $O/iter_base.err; exit 1; }
RAINGUN_HIP_LIB=$L/lhi/libraingun_hip.so timeout -k 10 120 python -u scripts/iter_stats.py synth1024 > $O/iter_lh.json 2> $O/iter_lh.err || { tail -5 $O/iter_lh.err; exit 1; }
cat $O/iter_base.json $O/iter_lh.json
RAINGUN_HIP_LIB=$L/lh/libraingun_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/pytest_lh.log 2>&1 || { tail -30 $O/pytest_lh.log; exit 1; }
tail -1 $O/pytest_lh.log
echo "== synth1024 steps 20"
bash scripts/ab_bench.sh "--workload synth1024 --no-extra --steps 20 --warmup 5" 3 abvar/base/libraingun_hip.so abvar/lh/libraingun_hip.so || exit 1
for S in 20 200; do
  echo "== test1 steps $S"
  bash scripts/ab_bench.sh "--workload test1 --no-extra --steps $S --warmup 5" 2 abvar/base/libraingun_hip.so abvar/up/libraingun_hip.so abvar/tp/libraingun_hip.so || exit 1
done
echo "== test3 steps 20"
bash scripts/ab_bench.sh "--workload test3 --no-extra --steps 20 --warmup 5" 2 abvar/base/libraingun_hip.so abvar/up/libraingun_hip.so abvar/tp/libraingun_hip.so || exit 1
echo "== host_visible pageable"
bash scripts/ab_bench.sh "--workload test1 --extra host_visible --steps 40 --warmup 5" 2 abvar/base/libraingun_hip.so abvar/cnt/libraingun_hip.so > $O/ab_hv.txt || exit 1
for f in gpurun_out/ab/abvar_base_*.json gpurun_out/ab/abvar_cnt_*.json; do
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);h=d.get('host_visible');print(sys.argv[1].split('/')[-1], h and (h['pinned']['ms_per_step'], h['pageable']['ms_per_step']))" $f
done
echo session done
