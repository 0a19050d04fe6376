#!/bin/bash
# LDS-side counters of the north-star timed configuration (one --pmc pass each)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; W=${1:-synth1024}; OUT=$R/gpurun_out/pmclds/$W; mkdir -p $OUT; export TMPDIR=/tmp; cd /tmp
BENCH="$R/bench.py --workload $W --no-extra --no-cpu-baseline --roofline-frames 1 --steps 3 --warmup 1"
i=0
for pass in "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 $BENCH > $OUT/p$i.log 2>&1
  echo "$W pass $i rc=$?"
done
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
for f in sorted(glob.glob(sys.argv[1] + "/p*/run_counter_collection.csv")):
    tot = collections.defaultdict(float); n = set()
    for r in csv.DictReader(open(f)):
        if "rg_render_kernel" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] += float(r["Counter_Value"]); n.add(r.get("Dispatch_Id", r.get("Correlation_Id")))
    print(f.split("/")[-2], {k: round(v / max(1, len(n)) / 1e6, 3) for k, v in tot.items()}, "M per frame", len(n), "dispatches")
PY
