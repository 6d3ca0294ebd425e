#!/bin/bash
# HBM traffic of one 240 s decode per kernel family (two counter passes) vs algorithmic bytes
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rm -rf gpurun_out/pv_f gpurun_out/pv_w
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pv_f -o run -- python3 tools/prof_dit.py --forwards 0 --vae > gpurun_out/pv_f.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pv_w -o run -- python3 tools/prof_dit.py --forwards 0 --vae > gpurun_out/pv_w.log 2>&1 && \
python3 tools/pmc_vae.py $(find gpurun_out/pv_f -name "*.db" | head -1) $(find gpurun_out/pv_w -name "*.db" | head -1) gpurun_out/r04_pmc_vae_traffic.json > gpurun_out/r04_pmc_vae_traffic.txt 2>&1
rc=$?; cat gpurun_out/r04_pmc_vae_traffic.txt | tail -60; rm -rf gpurun_out/pv_f gpurun_out/pv_w; exit $rc
