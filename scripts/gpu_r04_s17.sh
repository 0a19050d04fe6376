#!/bin/bash
# Round-4 session 17: the -m gpu suite at HEAD; unwind preload (up) and
# tile-slot prefetch (tp) vs HEAD, interleaved (light scenes at 20 / 200
# frames, the north star at 20); the parity tests with the prefetch library;
# the pageable host-visible frame with non-temporal host copies (cnt).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_s17; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for W in test1 test3; do
  for S in 20 200; do
    echo "== $W steps $S"
    bash scripts/ab_bench.sh "--workload $W --no-extra --steps $S --warmup 5" 2 abvar/base/libraingun_hip.so abvar/up/libraingun_hip.so abvar/tp/libraingun_hip.so || exit 1
  done
done
echo "== synth1024 steps 20"
bash scripts/ab_bench.sh "--workload synth1024 --no-extra --steps 20 --warmup 5" 2 abvar/base/libraingun_hip.so abvar/up/libraingun_hip.so abvar/tp/libraingun_hip.so || exit 1
RAINGUN_HIP_LIB=$PWD/abvar/tp/libraingun_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py > $O/pytest_tp.log 2>&1 || { tail -20 $O/pytest_tp.log; exit 1; }
tail -1 $O/pytest_tp.log
echo "== host_visible pageable"
bash scripts/ab_bench.sh "--workload test1 --extra host_visible --steps 40 --warmup 5" 2 abvar/base/libraingun_hip.so abvar/cnt/libraingun_hip.so > $O/ab_hv.txt || exit 1
for f in gpurun_out/ab/abvar_*_libraingun_hip.so.*.json; do
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);h=d.get('host_visible');print(sys.argv[1].split('/')[-1], h and (h['pinned']['ms_per_step'], h['pageable']['ms_per_step']))" $f
done
echo session done
