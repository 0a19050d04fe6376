#!/bin/bash
# Round-5 session 7: state of every line at HEAD (light buffers v2) -- the default bench.py
# line, the single-launch latency probe (test1, north star, with the rg_render_multi
# rehearsal), executed-work PMC of the north star at the timed configuration; plus the light
# path's shadow-trace ablation (abvar/lnoshadow: shadow batches not traced; timing only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/r05_s7; mkdir -p $O
export TMPDIR=/tmp
echo "== test1 shadow ablation (light path)"
bash scripts/ab_bench.sh "--workload test1 --no-extra --steps 50 --warmup 5" 2 raingun_amd/libraingun_hip.so abvar/lnoshadow/libraingun_hip.so || exit 1
timeout -k 10 600 python bench.py > $O/bench_full.json 2> $O/bench_full.err || { tail -20 $O/bench_full.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench_full.json').read().strip().splitlines()[-1]);print('full', d['value'], d['ms_per_step'], d['kernel_ms'], d['roofline'].get('frac'), d['host_visible']['pinned']['ms_per_step'], d['host_visible']['pageable']['ms_per_step'], d['host_visible']['multi_8gpu_rehearsal']['projected_speedup_vs_1gpu'], d['host_visible_north_star']['ms_per_step'], d['host_visible_north_star']['multi_8gpu_rehearsal']['projected_speedup_vs_1gpu'], [(k, d[k]['ms_per_step']) for k in ('test3_4k','north_star_1024_spheres','north_star_1024_spheres_8k','synth4096_16k')])"
timeout -k 10 300 python scripts/latency_probe.py test1 synth1024 > $O/latency.json 2> $O/latency.err || { tail $O/latency.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/latency.json'));print(json.dumps({k:(v if not isinstance(v,dict) else {kk:vv for kk,vv in v.items() if 'share8_kernel' not in kk}) for k,v in d.items()})[:1500])"
bash scripts/pmc_work.sh synth1024 3840 2160 20 || exit 1
echo session done
