#!/bin/bash
# Round-5 session 2: LightFrames variants against the pre-change library (abvar/base):
# in-tree = colour slots + kinds in LDS, refraction extras in the scratch Frame array;
# abvar/lfr_g = extras in a global buffer (session 1's library).  test1 200 / 20 frames,
# test3 50, the single-launch share latency; the GPU suite on the in-tree library first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05_s2; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_fullsize.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B=abvar/base/libraingun_hip.so; N=raingun_amd/libraingun_hip.so; G=abvar/lfr_g/libraingun_hip.so
for S in 200 20; do
  echo "== test1 steps $S"
  bash scripts/ab_bench.sh "--workload test1 --no-extra --steps $S --warmup 5" 3 $B $N $G || exit 1
done
echo "== test3 steps 50"
bash scripts/ab_bench.sh "--workload test3 --no-extra --steps 50 --warmup 5" 2 $B $N $G || exit 1
for L in $B $N; do
  tag=$(basename $(dirname $L))
  RAINGUN_HIP_LIB=$PWD/$L timeout -k 10 300 python scripts/latency_probe.py --no-multi test1 > $O/lat_$tag.json 2> $O/lat_$tag.err || { tail $O/lat_$tag.err; exit 1; }
  echo "latency $tag: $(python3 -c "import json;d=json.load(open('$O/lat_$tag.json'));t=d['test1'];print(t['whole_kernel_ms'], t['share8_max_ms'])")"
done
echo session done
