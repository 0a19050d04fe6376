#!/bin/bash
# One GPU session: parity tests, smoke, default bench (test1 + north-star synth1024),
# rocprof kernel-trace stats for both workloads.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo BENCH_FAILED; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
for W in test1 synth1024; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$W -o run --output-format csv -- python3 $R/bench.py --workload $W --steps 10 --warmup 2 --no-cpu-baseline --no-north-star --frames-in-flight 1 > $R/gpurun_out/prof_$W.log 2>&1 || { echo PROF_FAILED; tail -20 $R/gpurun_out/prof_$W.log; exit 1; }
  head -2 $R/gpurun_out/prof_$W/run_kernel_stats.csv
done
