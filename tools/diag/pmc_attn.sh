#!/bin/bash
# SQ counter passes over one attention shape: instruction mix + stall breakdown.
# usage: tools/diag/pmc_attn.sh <full|band|cross>
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
S=$1; O=gpurun_out/pmca_${S}
rm -rf $O; mkdir -p $O
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_WAVES --kernel-trace -d $O/a -o run -- python3 tools/diag/attn_one.py $S > $O/a.log 2>&1 && \
timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_TRANS_F32 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $O/b -o run -- python3 tools/diag/attn_one.py $S > $O/b.log 2>&1 && \
python3 tools/pmc_sq.py $(find $O/a -name "*.db" | head -1) $O/a.json > $O/a.txt && \
python3 tools/pmc_sq.py $(find $O/b -name "*.db" | head -1) $O/b.json > $O/b.txt
rc=$?
rm -rf $O/a $O/b
exit $rc
