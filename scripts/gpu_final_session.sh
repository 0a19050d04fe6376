#!/bin/bash
# Round-end measurement session: default bench line (every extra line, CPU baseline), its
# rocprofv3 kernel-trace summary, then the executed-work PMC of every bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -20 gpurun_out/bench_full.err; exit 1; }
tail -c 600 gpurun_out/bench_full.json; echo
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_default -o run -- python3 $R/bench.py --no-extra --no-cpu-baseline) > gpurun_out/prof_default.log 2>&1 || { tail -5 gpurun_out/prof_default.log; exit 1; }
head -3 gpurun_out/prof_default/run_kernel_stats.csv | cut -c1-160
bash scripts/pmc_all.sh
