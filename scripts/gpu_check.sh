set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/bench_test1.json 2> gpurun_out/bench_test1.err || { echo BENCH_FAILED; tail -30 gpurun_out/bench_test1.err; exit 1; }
cat gpurun_out/bench_test1.json
timeout -k 10 300 python bench.py --workload synth1024 --no-cpu-baseline > gpurun_out/bench_synth.json 2> gpurun_out/bench_synth.err || { echo BENCH2_FAILED; tail -30 gpurun_out/bench_synth.err; exit 1; }
cat gpurun_out/bench_synth.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_test1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_test1.log 2>&1 || { echo PROF_FAILED; tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_test1.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/prof_test1 -name '*stats*' | head
