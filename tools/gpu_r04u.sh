#!/bin/bash
# SwiGLU tail as one round of 128x256 two-phase ping-pong tiles (ACEHIP_GEMM_TAIL=1)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dit.py -k "gemm_variants" > gpurun_out/r04u_tests.log 2>&1 || { tail -30 gpurun_out/r04u_tests.log; exit 1; }
tail -2 gpurun_out/r04u_tests.log
SHAPES=swiglu_prod AB_KNOBS="ACEHIP_GEMM_TAIL=1" timeout -k 10 300 python -u tools/ab_gemm.py > gpurun_out/r04u_ab_gemm.log 2>&1 || { tail -20 gpurun_out/r04u_ab_gemm.log; exit 1; }
cat gpurun_out/r04u_ab_gemm.log
ROUNDS=3 timeout -k 10 400 python -u tools/ab_env_song.py 'ACEHIP_GEMM_TAIL=0' 'ACEHIP_GEMM_TAIL=1' > gpurun_out/r04u_ab_song.log 2>&1 || { tail -20 gpurun_out/r04u_ab_song.log; exit 1; }
cat gpurun_out/r04u_ab_song.log
