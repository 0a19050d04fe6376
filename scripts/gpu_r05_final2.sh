#!/bin/bash
# Round-5 measurement session at HEAD: the whole -m gpu suite and smoke(), the default bench
# line (every
# extra line, CPU baseline), the driver's configuration (--steps 20 --warmup 5)
# and the rocprofv3 kernel-trace summary of the default main line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; O=$R/gpurun_out/r05_final2; mkdir -p "$O"; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > "$O/pytest.log" 2>&1 || { tail -30 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { tail "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
timeout -k 10 600 python bench.py > "$O/bench_full.json" 2> "$O/bench_full.err" || { tail -20 "$O/bench_full.err"; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_full.json').read().strip().splitlines()[-1]);print('full', d['value'], d['ms_per_step'], d['kernel_ms'], d['roofline'].get('frac'), d['host_visible']['pinned']['ms_per_step'], d['host_visible']['pageable']['ms_per_step'], d['host_visible']['multi_8gpu_rehearsal']['projected_speedup_vs_1gpu'], d['host_visible_north_star']['multi_8gpu_rehearsal']['projected_speedup_vs_1gpu'], d['north_star_1024_spheres']['ms_per_step'])"
for k in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-extra > "$O/bench_driver_cfg$k.json" 2> "$O/bench_driver_cfg$k.err" || { tail -20 "$O/bench_driver_cfg$k.err"; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_driver_cfg$k.json').read().strip().splitlines()[-1]);print('driver-cfg', d['value'], d['ms_per_step'])"
done
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_default" -o run -- python3 "$R/bench.py" --no-extra --no-cpu-baseline) > "$O/prof_default.log" 2>&1 || { tail -5 "$O/prof_default.log"; exit 1; }
head -3 "$O/prof_default/run_kernel_stats.csv" | cut -c1-160
echo session done
