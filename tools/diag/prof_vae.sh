#!/bin/bash
# kernel-trace stats + SQ counters of one full-size decode (tools/diag/vae_one.py)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/profv
rm -rf $O; mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/k -o run -- python3 tools/diag/vae_one.py 2 > $O/k.log 2>&1 && \
python3 tools/rocprof_summary.py $(find $O/k -name "*.db" | head -1) > $O/kernel_stats.md && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_WAVES --kernel-trace -d $O/a -o run -- python3 tools/diag/vae_one.py > $O/a.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d $O/b -o run -- python3 tools/diag/vae_one.py > $O/b.log 2>&1 && \
python3 tools/pmc_sq.py $(find $O/a -name "*.db" | head -1) $O/a.json > $O/a.txt && \
python3 tools/pmc_sq.py $(find $O/b -name "*.db" | head -1) $O/b.json > $O/b.txt
rc=$?
rm -rf $O/k $O/a $O/b
exit $rc
