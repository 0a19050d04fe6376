#!/bin/bash
# Round-4 session 25: leaf prefetch on global sphere tables as the default
# (in-tree library) against the previous HEAD (abvar/base2): the whole -m gpu
# suite, the configs[4] shape at 1080p and the configs[4] bench line at 16K,
# the north star (unchanged kernel code) as a control.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r04_s25; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
echo "== synth4096p8d8 1920x1080 steps 5"
bash scripts/ab_bench.sh "--workload synth4096p8d8 --width 1920 --height 1080 --no-extra --steps 5 --warmup 2" 3 abvar/base2/libraingun_hip.so raingun_amd/libraingun_hip.so || exit 1
echo "== configs[4] line (16K)"
for lib in abvar/base2/libraingun_hip.so raingun_amd/libraingun_hip.so; do
  RAINGUN_HIP_LIB=$PWD/$lib timeout -k 10 400 python -u bench.py --workload test1 --extra synth4096_16k --steps 5 --warmup 2 --no-cpu-baseline > $O/c4_$(basename $(dirname $lib)).json 2> $O/c4.err || { tail -5 $O/c4.err; exit 1; }
  python3 -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);x=d['synth4096_16k'];print(sys.argv[1], x['ms_per_step'], x['value'])" $O/c4_$(basename $(dirname $lib)).json
done
echo "== synth1024 steps 20"
bash scripts/ab_bench.sh "--workload synth1024 --no-extra --steps 20 --warmup 5" 2 abvar/base2/libraingun_hip.so raingun_amd/libraingun_hip.so || exit 1
echo session done
