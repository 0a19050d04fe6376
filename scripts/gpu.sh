#!/bin/bash
# One parameterised GPU session runner (replaces the per-session scripts of rounds 4-5,
# which live in git history before round 6).  Every step runs under its own time limit;
# the first failing step ends the session (no retries).  Output under gpurun_out/$TAG/.
#
#   bash scripts/gpu.sh TAG step [step ...]
#
# steps (arguments separated by ':'; a space inside one step's bench args as ','):
#   tests[:selection]             pytest -m gpu (one process, per-test thread timeout)
#   smoke                         __graft_entry__.smoke()
#   bench[:args]                  bench.py (default: the driver configuration --steps 20 --warmup 5)
#   benchfull                     the default bench.py run (every line, CPU baseline)
#   trace[:args]                  rocprofv3 --kernel-trace --stats of bench.py --no-extra
#   ab:args:rounds:lib1,lib2..    interleaved A/B of library variants (scripts/ab_bench.sh)
#   pmc:wl:w:h:steps              executed-work PMC of one bench line (scripts/pmc_work.sh)
#   pmcall                        scripts/pmc_all.sh (every bench line)
#   pcsamp:wl[:interval]          stochastic PC sampling of bench.py's timed configuration
#   iter:lib:wl,wl..              RG_ITER_STATS counters (scripts/iter_stats.py) with a variant library
#   shares:wl,wl..                per-rank 1/8 shares (scripts/rank_shares.sh)
#   latency:wl,wl..[:lib]         single-launch latency + rg_render_multi rehearsal (scripts/latency_probe.py)
#   py:script:args                any repo python script (args ',' -> ' '), output to TAG/<script>.out
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
TAG=$1; shift
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp
log() { echo "[$(date +%H:%M:%S)] $*" | tee -a "$O/session.txt"; }
sp() { local x="${1//,/ }"; x="${x//@/::}"; x="${x//^/,}"; echo "${x//\~/:}"; }  # "," -> " ", "@" -> "::" (pytest node ids), "^" -> ",", "~" -> ":"

for step in "$@"; do
  IFS=':' read -r kind a1 a2 a3 a4 <<< "$step"
  log "step $step"
  case $kind in
    tests)
      timeout -k 10 900 python -u -m pytest -x -v --timeout 180 --timeout-method thread -m gpu $(sp "${a1:-tests/}") \
        > "$O/pytest.log" 2>&1
      rc=$?; tail -3 "$O/pytest.log" | tee -a "$O/session.txt"
      [ $rc -eq 0 ] || { grep -E "FAILED|Error" "$O/pytest.log" | head -20; exit $rc; } ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
        || { tail "$O/smoke.log"; exit 1; }
      tail -1 "$O/smoke.log" | tee -a "$O/session.txt" ;;
    bench)
      args=$(sp "${a1:---steps,20,--warmup,5}")
      n=$(ls "$O" | grep -c '^bench\.[0-9]*\.json$')
      timeout -k 10 400 python bench.py $args > "$O/bench.$n.json" 2> "$O/bench.$n.err" \
        || { tail -20 "$O/bench.$n.err"; exit 1; }
      python - "$O/bench.$n.json" "$args" <<'PY' | tee -a "$O/session.txt"
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
extra = {k: v["ms_per_step"] for k, v in d.items() if isinstance(v, dict) and "ms_per_step" in v}
print("bench", sys.argv[2], "ms", d["ms_per_step"], "frac", d.get("roofline", {}).get("frac"), json.dumps(extra))
PY
      ;;
    benchfull)
      timeout -k 10 600 python bench.py > "$O/bench_full.json" 2> "$O/bench_full.err" \
        || { tail -20 "$O/bench_full.err"; exit 1; }
      tail -c 400 "$O/bench_full.json" | tee -a "$O/session.txt"; echo ;;
    trace)
      args=$(sp "${a1:---steps,20,--warmup,5}")
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/trace" -o run -- \
        python3 "$R/bench.py" --no-extra --no-cpu-baseline $args) > "$O/trace.log" 2>&1 \
        || { tail -5 "$O/trace.log"; exit 1; }
      head -4 "$O/trace/run_kernel_stats.csv" | cut -c1-200 | tee -a "$O/session.txt" ;;
    ab)
      libs=$(sp "$a3")
      bash scripts/ab_bench.sh "$(sp "$a1")" "$a2" $libs 2>&1 | tee -a "$O/session.txt"
      rc=${PIPESTATUS[0]}; cp -r gpurun_out/ab "$O/ab" 2>/dev/null; rm -rf gpurun_out/ab
      [ $rc -eq 0 ] || exit $rc ;;
    pmc)
      bash scripts/pmc_work.sh "$a1" "$a2" "$a3" "$a4" 2>&1 | tee -a "$O/session.txt"
      [ ${PIPESTATUS[0]} -eq 0 ] || exit 1 ;;
    pmcall)
      bash scripts/pmc_all.sh 2>&1 | tee -a "$O/session.txt"
      [ ${PIPESTATUS[0]} -eq 0 ] || exit 1 ;;
    pcsamp)
      wl=${a1:-test1}; iv=${a2:-1048576}
      (cd /tmp && timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic \
        --pc-sampling-unit cycles --pc-sampling-interval "$iv" --output-format csv -d "$O/pcs_$wl" -o run -- \
        python3 "$R/bench.py" --workload "$wl" --no-extra --no-cpu-baseline --roofline-frames 1 --steps 40 --warmup 2) \
        > "$O/pcs_$wl.log" 2>&1 || { tail -20 "$O/pcs_$wl.log"; exit 1; }
      ls -la "$O/pcs_$wl" | tee -a "$O/session.txt" ;;
    iter)
      for wl in $(sp "$a2"); do
        RAINGUN_HIP_LIB=$R/$a1 timeout -k 10 200 python scripts/iter_stats.py $wl >> "$O/iter.jsonl" 2> "$O/iter.err" \
          || { tail "$O/iter.err"; exit 1; }
      done
      cat "$O/iter.jsonl" | tee -a "$O/session.txt" ;;
    shares)
      bash scripts/rank_shares.sh $(sp "$a1") 2>&1 | tee -a "$O/session.txt"
      rc=${PIPESTATUS[0]}; cp -r gpurun_out/shares "$O/shares" 2>/dev/null; rm -rf gpurun_out/shares
      [ $rc -eq 0 ] || exit $rc ;;
    latency)
      tag=lat${a2:+_$(basename "$(dirname "$a2")")}
      RAINGUN_HIP_LIB=${a2:+$R/$a2} timeout -k 10 300 python scripts/latency_probe.py $(sp "$a1") > "$O/$tag.json" \
        2> "$O/$tag.err" || { tail "$O/$tag.err"; exit 1; }
      python - "$O/$tag.json" "$tag" <<'PY' | tee -a "$O/session.txt"
import json, sys
D = json.load(open(sys.argv[1]))
for wl, d in D.items():
    if isinstance(d, dict) and "share8_max_ms" in d:
        m = d.get("multi_8gpu_rehearsal", {})
        print(sys.argv[2], wl, "whole", d["whole_kernel_ms"], "share8_max", d["share8_max_ms"], "pinned1", d.get("host_pinned_1gpu_ms"),
              "multi", m.get("projected_ms_per_step"), m.get("projected_speedup_vs_1gpu"), m.get("per_device_ms"))
PY
      ;;
    py)
      base=$(basename "$a1" .py)$(echo "${a2:+_$a2}" | tr -c 'A-Za-z0-9_\n' '_' | cut -c1-40)
      timeout -k 10 400 python "$a1" $(sp "$a2") > "$O/$base.out" 2> "$O/$base.err" \
        || { tail -20 "$O/$base.err"; exit 1; }
      tail -c 1500 "$O/$base.out" | tee -a "$O/session.txt"; echo ;;
    *) echo "unknown step $kind"; exit 2 ;;
  esac
done
log "session done"
