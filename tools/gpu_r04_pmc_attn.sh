#!/bin/bash
# SQ counter passes (waves, wait / issue split, MFMA busy) of the 240 s attention launches:
# band (persistent and one workgroup per unit), full, cross of the conditional rows
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
C="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
run() {   # tag shape env...
  local tag=$1 shape=$2; shift 2
  rm -rf gpurun_out/pa_$tag
  env "$@" timeout -s KILL 90 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pa_$tag -o run -- python3 tools/attn_once.py $shape 10 > gpurun_out/pa_$tag.log 2>&1 || { tail -5 gpurun_out/pa_$tag.log; exit 1; }
  python3 tools/pmc_sq.py $(find gpurun_out/pa_$tag -name "*.db" | head -1) gpurun_out/r04_pmc_attn_$tag.json > /dev/null || exit 1
  rm -rf gpurun_out/pa_$tag
  echo "$tag"; cat gpurun_out/r04_pmc_attn_$tag.json
}
run band_persist band ACEHIP_ATTN_PERSIST=1
run band_unit band ACEHIP_ATTN_PERSIST=0
run full full ACEHIP_ATTN_PW=2
run cross1 cross1 ACEHIP_ATTN_PW=2
