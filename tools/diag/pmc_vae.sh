#!/bin/bash
# SQ counter passes over one full-size VAE decode: stall breakdown, instruction mix, LDS conflicts.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/pmcv
rm -rf $O; mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_WAVES --kernel-trace -d $O/a -o run -- python3 tools/diag/vae_one.py > $O/a.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $O/b -o run -- python3 tools/diag/vae_one.py > $O/b.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAVES --kernel-trace -d $O/c -o run -- python3 tools/diag/vae_one.py > $O/c.log 2>&1 && \
python3 tools/pmc_sq.py $(find $O/a -name "*.db" | head -1) $O/a.json > $O/a.txt && \
python3 tools/pmc_sq.py $(find $O/b -name "*.db" | head -1) $O/b.json > $O/b.txt && \
python3 tools/pmc_sq.py $(find $O/c -name "*.db" | head -1) $O/c.json > $O/c.txt
rc=$?
rm -rf $O/a $O/b $O/c
exit $rc
