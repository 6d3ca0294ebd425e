#!/bin/bash
# SQ counter passes on the full-attention shape, both kernels (ACEHIP_ATTN_PW 0 / 7)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
C1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE"
for pw in 0 7; do
  rm -rf gpurun_out/pa$pw
  ACEHIP_ATTN_PW=$pw timeout -s KILL 90 rocprofv3 --pmc $C1 --kernel-trace -d gpurun_out/pa$pw -o run -- python3 tools/attn_once.py ${SHAPE:-full} 10 > gpurun_out/pa$pw.log 2>&1 || { tail -5 gpurun_out/pa$pw.log; exit 1; }
  python3 tools/pmc_sq.py $(find gpurun_out/pa$pw -name "*.db" | head -1) gpurun_out/pmc_attn_pw$pw.json > gpurun_out/pmc_attn_pw$pw.txt || exit 1
  rm -rf gpurun_out/pa$pw
done
cat gpurun_out/pmc_attn_pw0.json gpurun_out/pmc_attn_pw7.json
