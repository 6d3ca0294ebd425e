#!/bin/bash
# helper waves in the two-phase ping-pong tiles (variants 14 = 192x256, 15 = 128x256)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dit.py -k "gemm_variants" > gpurun_out/r04v_tests.log 2>&1 || { tail -30 gpurun_out/r04v_tests.log; exit 1; }
tail -2 gpurun_out/r04v_tests.log
SHAPES=down,qkv,o AB_VARIANTS=14 timeout -k 10 300 python -u tools/ab_gemm.py > gpurun_out/r04v_ab_gemm.log 2>&1 || { tail -20 gpurun_out/r04v_ab_gemm.log; exit 1; }
cat gpurun_out/r04v_ab_gemm.log
