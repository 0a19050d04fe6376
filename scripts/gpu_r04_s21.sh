#!/bin/bash
# Round-4 session 21: per-lane walk with helpers after the fence fix (lh2*):
# parity, walk statistics, north star A/B + single-launch share latency; then
# the light-path knobs (unwind preload up / tile-slot prefetch tp) and
# non-temporal pageable host copies (cnt) against HEAD.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_s21; mkdir -p $O
L=$PWD/abvar
lh_ok=1
for v in lh2 lh2r3; do
  RAINGUN_HIP_LIB=$L/$v/libraingun_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/pytest_$v.log 2>&1
  rc=$?
  echo "$v rc=$rc: $(tail -1 $O/pytest_$v.log)"
  if [ $rc -eq 1 ]; then lh_ok=0; grep -m5 "^E \|^FAILED" $O/pytest_$v.log; break; fi
  [ $rc -ne 0 ] && exit 1
done
if [ $lh_ok -eq 1 ]; then
  RAINGUN_HIP_LIB=$L/lhi2/libraingun_hip.so timeout -k 10 120 python -u scripts/iter_stats.py synth1024 > $O/iter_lh2.json 2> $O/iter_lh2.err || { tail -5 $O/iter_lh2.err; exit 1; }
  cat $O/iter_lh2.json
  echo "== synth1024 steps 20"
  bash scripts/ab_bench.sh "--workload synth1024 --no-extra --steps 20 --warmup 5" 2 abvar/base/libraingun_hip.so abvar/lh2/libraingun_hip.so abvar/lh2a24/libraingun_hip.so abvar/lh2a52/libraingun_hip.so abvar/lh2r3/libraingun_hip.so || exit 1
  for v in base lh2 lh2r3; do
    RAINGUN_HIP_LIB=$L/$v/libraingun_hip.so timeout -k 10 300 python -u scripts/latency_probe.py synth1024 > $O/latency_$v.json 2> $O/latency_$v.err || { tail -5 $O/latency_$v.err; exit 1; }
    python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[1], json.dumps(d)[:700])" $O/latency_$v.json
  done
fi
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
