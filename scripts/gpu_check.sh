#!/bin/bash
# One GPU session: parity tests, smoke, bench (both workloads), rocprof kernel trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$PWD
timeout -k 10 600 python -m pytest tests/ -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAILED; tail -20 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log | tail -1
timeout -k 10 300 python bench.py > gpurun_out/bench_test1.json 2> gpurun_out/bench_test1.err || { echo BENCH_FAILED; tail -30 gpurun_out/bench_test1.err; exit 1; }
cat gpurun_out/bench_test1.json
timeout -k 10 400 python bench.py --workload synth1024 > gpurun_out/bench_synth.json 2> gpurun_out/bench_synth.err || { echo BENCH2_FAILED; tail -30 gpurun_out/bench_synth.err; exit 1; }
cat gpurun_out/bench_synth.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_test1 -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_test1.log 2>&1 || { echo PROF_FAILED; tail -20 $R/gpurun_out/prof_test1.log; exit 1; }
cat $R/gpurun_out/prof_test1/run_kernel_stats.csv | head -3
