#!/bin/bash
# 96x256 one-interval ping-pong (variant 12) at the half-chip shapes
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dit.py -k "gemm_variants" > gpurun_out/r04q_tests.log 2>&1 || { tail -30 gpurun_out/r04q_tests.log; exit 1; }
tail -2 gpurun_out/r04q_tests.log
SHAPES=o_half,crossq AB_VARIANTS=14,15 timeout -k 10 300 python -u tools/ab_gemm.py > gpurun_out/r04q_ab_gemm.log 2>&1 || { tail -20 gpurun_out/r04q_ab_gemm.log; exit 1; }
cat gpurun_out/r04q_ab_gemm.log
