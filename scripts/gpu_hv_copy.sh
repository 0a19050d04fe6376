#!/bin/bash
# Host-visible test1 frames (pinned, banded): band copies by the runtime's blit copy vs a small copy
# grid, and CU-masked copy / render streams.  ms per rg_render_image call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/hvc
run() {  # label, env..., then bands
  local label=$1; shift
  env "$@" timeout -k 10 120 python3 scripts/hv_timeline.py ${HVC_WL:-test1} ${HVC_BANDS:-0} > gpurun_out/hvc/$label.log 2>&1 || { echo "FAIL $label"; tail -5 gpurun_out/hvc/$label.log; exit 1; }
  echo "$label $(grep 'ms per frame' gpurun_out/hvc/$label.log)"
}
run base X=0
run blk16 RG_HV_COPY_BLOCKS=16
run blk32 RG_HV_COPY_BLOCKS=32
run blk64 RG_HV_COPY_BLOCKS=64
run cus16 RG_HV_COPY_CUS=16
run cus32 RG_HV_COPY_CUS=32
run cus16c RG_HV_COPY_CUS=16 RG_HV_CUPAT=1
run cus32x RG_HV_COPY_CUS=32 RG_HV_RENDER_EXCL=1
run cus16x RG_HV_COPY_CUS=16 RG_HV_RENDER_EXCL=1
run cus32xb32 RG_HV_COPY_CUS=32 RG_HV_RENDER_EXCL=1 RG_HV_COPY_BLOCKS=32
run cus16xb16 RG_HV_COPY_CUS=16 RG_HV_RENDER_EXCL=1 RG_HV_COPY_BLOCKS=16
run base2 X=0
