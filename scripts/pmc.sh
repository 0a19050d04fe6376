#!/bin/bash
# PMC passes for one bench workload: bash scripts/pmc.sh <workload> [steps]
# Each pass: --pmc <counters> --kernel-trace only (no sys/runtime traces).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD; W=${1:-test1}; STEPS=${2:-3}
mkdir -p gpurun_out/pmc_$W
export TMPDIR=/tmp
cd /tmp
i=0
shift 2 || true
for pass in "FETCH_SIZE" "WRITE_SIZE" \
            "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS" \
            "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
            "SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64" \
            "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d $R/gpurun_out/pmc_$W/p$i -o run -- python3 $R/bench.py --workload $W --steps $STEPS --warmup 1 --no-cpu-baseline --no-north-star --frames-in-flight 1 > $R/gpurun_out/pmc_$W/p$i.log 2>&1
  rc=$?
  echo "pass $i [$pass] rc=$rc"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then echo "stopping"; exit $rc; fi
done
