#!/bin/bash
# two-phase ping-pong schedule (variants 9 / 10): correctness, then one-process A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dit.py -k "gemm_variants or pingpong or residual" > gpurun_out/r04g_tests.log 2>&1 || { tail -30 gpurun_out/r04g_tests.log; exit 1; }
tail -3 gpurun_out/r04g_tests.log
SHAPES=down,o AB_KNOBS="ACEHIP_GEMM_PFRES=1" timeout -k 10 400 python -u tools/ab_gemm.py > gpurun_out/r04g_ab_gemm.log 2>&1 || { tail -20 gpurun_out/r04g_ab_gemm.log; exit 1; }
cat gpurun_out/r04g_ab_gemm.log
