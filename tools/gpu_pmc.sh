#!/bin/bash
# PMC passes (separate runs per counter group, kernel-trace only), per MI355X_MICROARCH.md §HBM
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run -- python3 tools/prof_dit.py --forwards 1 --vae > gpurun_out/pmc1.log 2>&1 || { tail -20 gpurun_out/pmc1.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run -- python3 tools/prof_dit.py --forwards 1 --vae > gpurun_out/pmc2.log 2>&1 || { tail -20 gpurun_out/pmc2.log; exit 1; }
ls -R gpurun_out/pmc_fetch | head
