#!/bin/bash
# Round-4 session 22: tile-slot prefetch as the default (in-tree library):
# the whole -m gpu suite and smoke on it; north star and test1 A/B against the
# previous default (abvar/base) and with the unwind preload on top (tpup); the
# default bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_s22; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
echo "== synth1024 steps 20"
bash scripts/ab_bench.sh "--workload synth1024 --no-extra --steps 20 --warmup 5" 3 abvar/base/libraingun_hip.so raingun_amd/libraingun_hip.so || exit 1
echo "== test1 steps 200"
bash scripts/ab_bench.sh "--workload test1 --no-extra --steps 200 --warmup 5" 2 abvar/base/libraingun_hip.so raingun_amd/libraingun_hip.so abvar/tpup/libraingun_hip.so || exit 1
echo "== test1 steps 20"
bash scripts/ab_bench.sh "--workload test1 --no-extra --steps 20 --warmup 5" 2 abvar/base/libraingun_hip.so raingun_amd/libraingun_hip.so abvar/tpup/libraingun_hip.so || exit 1
timeout -k 10 600 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
cat $O/bench_default.json
echo session done
