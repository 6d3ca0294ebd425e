#!/bin/bash
# persistent ping-pong GEMM (ACEHIP_GEMM_PERSIST): parity, kernel A/B, song A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dit.py tests/test_gpu_fused.py -k "gemm or headpost" > gpurun_out/r04p2_tests.log 2>&1 || { tail -30 gpurun_out/r04p2_tests.log; exit 1; }
tail -2 gpurun_out/r04p2_tests.log
SHAPES=swiglu_prod,qkv,swiglu AB_KNOBS="ACEHIP_GEMM_PERSIST=1" timeout -k 10 400 python -u tools/ab_gemm.py tools/ab/libacehip_head.so > gpurun_out/r04p2_ab_gemm.log 2>&1 || { tail -20 gpurun_out/r04p2_ab_gemm.log; exit 1; }
cat gpurun_out/r04p2_ab_gemm.log
timeout -k 10 300 python -u tools/ab_headpost.py > gpurun_out/r04p2_ab_hp0.log 2>&1 || { tail -20 gpurun_out/r04p2_ab_hp0.log; exit 1; }
ACEHIP_GEMM_PERSIST=1 timeout -k 10 300 python -u tools/ab_headpost.py > gpurun_out/r04p2_ab_hp1.log 2>&1 || { tail -20 gpurun_out/r04p2_ab_hp1.log; exit 1; }
tail -1 gpurun_out/r04p2_ab_hp0.log; tail -1 gpurun_out/r04p2_ab_hp1.log
ROUNDS=4 timeout -k 10 400 python -u tools/ab_env_song.py 'ACEHIP_GEMM_PERSIST=0' 'ACEHIP_GEMM_PERSIST=1' > gpurun_out/r04p2_ab_song.log 2>&1 || { tail -20 gpurun_out/r04p2_ab_song.log; exit 1; }
cat gpurun_out/r04p2_ab_song.log
