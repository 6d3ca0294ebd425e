#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
SHAPES=o_half,crossq AB_VARIANTS=0,13,20,21,22 timeout -k 10 300 python -u tools/ab_gemm.py > gpurun_out/r04e_ab_gemm.log 2>&1 || { tail -20 gpurun_out/r04e_ab_gemm.log; exit 1; }
cat gpurun_out/r04e_ab_gemm.log
SHAPES=down,o timeout -k 10 300 python -u tools/ab_gemm.py tools/ab/libacehip_pfres.so > gpurun_out/r04e_ab_pfres.log 2>&1 || { tail -20 gpurun_out/r04e_ab_pfres.log; exit 1; }
cat gpurun_out/r04e_ab_pfres.log
