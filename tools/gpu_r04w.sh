#!/bin/bash
# helper waves as the default for the 192 / 128-row two-phase tiles: GEMM tests, A/B 2 vs 4 helpers, song A/B
set -o pipefail
mkdir -p gpurun_out
#timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dit.py tests/test_gpu_fused.py -k "gemm or headpost" > gpurun_out/r04w_tests.log 2>&1 || { tail -30 gpurun_out/r04w_tests.log; exit 1; }
#tail -2
#SHAPES=down,qkv,o,swiglu_prod AB_VARIANTS=14 AB_KNOBS="ACEHIP_GEMM_HELPERS=0" timeout -k 10 400 python -u tools/ab_gemm.py > gpurun_out/r04w_ab_gemm.log 2>&1 || { tail -20 gpurun_out/r04w_ab_gemm.log; exit 1; }
#cat
ROUNDS=4 timeout -k 10 400 python -u tools/ab_env_song.py 'ACEHIP_GEMM_HELPERS=0' 'ACEHIP_GEMM_HELPERS=1' 'ACEHIP_GEMM_HELPERS=3' > gpurun_out/r04x_ab_song.log 2>&1 || { tail -20 gpurun_out/r04x_ab_song.log; exit 1; }
cat gpurun_out/r04x_ab_song.log
