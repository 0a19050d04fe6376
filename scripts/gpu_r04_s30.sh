#!/bin/bash
# Round-4 session 30: single-launch evidence at HEAD -- the rocprofv3 kernel
# trace of the latency probe (whole frames and 1/8 shares of test1 and the north
# star, one launch at a time) and per-wave timelines of test1 (RG_WAVE_TIMES).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/r04_s30; mkdir -p $O; export TMPDIR=/tmp
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_latency" -o run -- python3 "$R/scripts/latency_probe.py" --no-multi test1 synth1024) > $O/latency_probe.json 2> $O/latency_probe.err || { tail -5 $O/latency_probe.err; exit 1; }
head -4 $O/prof_latency/run_kernel_stats.csv | cut -c1-200
RAINGUN_HIP_LIB=$R/abvar/wt/libraingun_hip.so timeout -k 10 300 python -u scripts/wave_times.py test1 > $O/wave_times.json 2> $O/wave_times.err || { tail -5 $O/wave_times.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/wave_times.json'))
for k,v in d['test1'].items(): print(k, v['kernel_ms'], v['waves'], 'life', v['life_us_p0_10_50_90_99_100'], 'end', v['end_us_p0_10_50_90_99_100'][-1], 'tiles', v['tiles_per_wave_p0_50_100'])"
echo session done
