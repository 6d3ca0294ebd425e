#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/ab_gemm.py tools/ab/libacehip_spl4.so > gpurun_out/r04d_ab_gemm.log 2>&1 || { tail -20 gpurun_out/r04d_ab_gemm.log; exit 1; }
cat gpurun_out/r04d_ab_gemm.log
