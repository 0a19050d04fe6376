#!/bin/bash
# session 29: round delta, round-4 HEAD 197b0cb (abvar/r04) vs round-5 HEAD, same box, interleaved
set -e
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/s29
L="abvar/r04/libraingun_hip.so raingun_amd/libraingun_hip.so"
echo "== test1 4K, 200 frames"
bash scripts/ab_bench.sh "--workload test1 --no-extra --steps 200 --warmup 5" 3 $L
echo "== test1 4K, driver configuration (20 frames)"
bash scripts/ab_bench.sh "--workload test1 --no-extra --steps 20 --warmup 5" 3 $L
echo "== test3 4K, 100 frames"
bash scripts/ab_bench.sh "--workload test3 --no-extra --steps 100 --warmup 5" 2 $L
echo "== north star 4K, 200 frames"
bash scripts/ab_bench.sh "--workload synth1024 --no-extra --steps 200 --warmup 5" 3 $L
echo "== north star 8K, 40 frames"
bash scripts/ab_bench.sh "--workload synth1024 --width 7680 --height 4320 --no-extra --steps 40 --warmup 3" 2 $L
echo "== configs[4] synth4096p8d8 16384x16384, 4 frames"
bash scripts/ab_bench.sh "--workload synth4096p8d8 --width 16384 --height 16384 --no-extra --steps 4 --warmup 1" 2 $L
echo "== host-visible lines"
for r in 1 2; do
for v in abvar/r04 raingun_amd; do
  RAINGUN_HIP_LIB=$PWD/$v/libraingun_hip.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --extra host_visible,host_visible_north_star > gpurun_out/s29/hv_$(basename $v).$r.json 2> gpurun_out/s29/hv_$(basename $v).$r.err
  python - gpurun_out/s29/hv_$(basename $v).$r.json $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
out = [sys.argv[2]]
for k in ("host_visible", "host_visible_north_star"):
    h = d[k]
    out.append(f"{k}: pinned {h['pinned']['ms_per_step']} pageable {h['pageable']['ms_per_step']} "
               f"multi {h['multi_8gpu_rehearsal']['projected_ms_per_step']} ({h['multi_8gpu_rehearsal']['projected_speedup_vs_1gpu']}x)")
print(" | ".join(out))
PY
done
done
echo "== single launches"
for v in abvar/r04 raingun_amd; do
  RAINGUN_HIP_LIB=$PWD/$v/libraingun_hip.so timeout -k 10 300 python scripts/latency_probe.py --no-multi test1 synth1024 > gpurun_out/s29/lat_$(basename $v).json 2> gpurun_out/s29/lat_$(basename $v).err
  python -c "
import json,sys
D=json.load(open(sys.argv[1]))
for wl in ('test1','synth1024'):
    d=D[wl]; print(sys.argv[2], wl, 'whole', d['whole_kernel_ms'], 'share8_max', d['share8_max_ms'])" gpurun_out/s29/lat_$(basename $v).json $v
done
