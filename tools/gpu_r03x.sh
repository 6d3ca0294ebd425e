#!/bin/bash
# small-M GEMM A/B (turbo shapes)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/bench_small_m.py > gpurun_out/r03x_small_m.log 2>&1 || { tail -20 gpurun_out/r03x_small_m.log; exit 1; }
cat gpurun_out/r03x_small_m.log
