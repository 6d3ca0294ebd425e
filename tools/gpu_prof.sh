#!/bin/bash
# Profiling pass on a GPU box (rocprofv3, MI355X_MICROARCH.md §rocprofv3):
#  1. kernel trace + --stats of a short bench run  -> gpurun_out/prof/
#  2. SQ/GRBM counter pass (MFMA busy, waits, effective clock) on tools/prof_dit.py
#  3. FETCH_SIZE and WRITE_SIZE passes (separate runs)
# Every step under its own timeout, chained with && (a failure ends the script).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
TAG=${TAG:-r02}
rm -rf gpurun_out/prof gpurun_out/pmc_sq gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || echo "counter list failed (ignored)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace -d gpurun_out/pmc_sq -o run -- python3 tools/prof_dit.py --forwards 1 --vae > gpurun_out/pmc_sq.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run -- python3 tools/prof_dit.py --forwards 1 --vae > gpurun_out/pmc_fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run -- python3 tools/prof_dit.py --forwards 1 --vae > gpurun_out/pmc_write.log 2>&1 && \
echo "prof ok" && \
python3 tools/rocprof_summary.py $(find gpurun_out/prof -name "*.db" | head -1) > gpurun_out/${TAG}_kernel_stats.md && \
python3 tools/pmc_sq.py $(find gpurun_out/pmc_sq -name "*.db" | head -1) gpurun_out/${TAG}_pmc_sq.json > gpurun_out/${TAG}_pmc_sq.txt && \
python3 tools/pmc_traffic.py $(find gpurun_out/pmc_fetch -name "*.db" | head -1) $(find gpurun_out/pmc_write -name "*.db" | head -1) gpurun_out/${TAG}_pmc_traffic.json > gpurun_out/${TAG}_pmc_traffic.txt
rc=$?
# the databases are large: keep only the summaries (gpurun copies back <= 64 MiB)
find gpurun_out/prof -name "*stats*" -exec cp {} gpurun_out/ \; 2>/dev/null
rm -rf gpurun_out/prof gpurun_out/pmc_sq gpurun_out/pmc_fetch gpurun_out/pmc_write
exit $rc
