#!/bin/bash
# Round-5 session 1: the light path's frames out of scratch (LightFrames).  The whole -m gpu
# suite, then interleaved A/Bs against the library before the change (abvar/base, built from
# 10583a3): test1 200 and 20 frames, test3; the single-launch latency of test1's shares; the
# executed-work PMC passes of test1 at the bench's timed configuration.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05_s1; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B=abvar/base/libraingun_hip.so; N=raingun_amd/libraingun_hip.so
for S in 200 20; do
  echo "== test1 steps $S"
  bash scripts/ab_bench.sh "--workload test1 --no-extra --steps $S --warmup 5" 3 $B $N || exit 1
done
echo "== test3 steps 50"
bash scripts/ab_bench.sh "--workload test3 --no-extra --steps 50 --warmup 5" 2 $B $N || exit 1
for L in $B $N; do
  tag=$(basename $(dirname $L))
  RAINGUN_HIP_LIB=$PWD/$L timeout -k 10 300 python scripts/latency_probe.py --no-multi test1 > $O/lat_$tag.json 2> $O/lat_$tag.err || { tail $O/lat_$tag.err; exit 1; }
  echo "latency $tag: $(python3 -c "import json;d=json.load(open('$O/lat_$tag.json'));print(json.dumps(d)[:400])")"
done
bash scripts/pmc_work.sh test1 3840 2160 20 || exit 1
echo session done
