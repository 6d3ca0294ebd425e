#!/bin/bash
# kernel trace of one 240 s decode on ru8_kernel (ACEHIP_RU7=2)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rm -rf gpurun_out/pvae
ACEHIP_RU7=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pvae -o run -- python3 tools/prof_dit.py --forwards 0 --vae > gpurun_out/pvae.log 2>&1 && python3 tools/rocprof_summary.py $(find gpurun_out/pvae -name "*.db" | head -1) > gpurun_out/r04ru8_vae_kernel_stats.md; rc=$?
rm -rf gpurun_out/pvae; head -30 gpurun_out/r04ru8_vae_kernel_stats.md; exit $rc
