#!/bin/bash
# snake 1/2π fold: VAE parity tests, decode A/B against HEAD
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_vae_units.py tests/test_vae.py -m gpu > gpurun_out/r04p_tests.log 2>&1 || { tail -30 gpurun_out/r04p_tests.log; exit 1; }
tail -2 gpurun_out/r04p_tests.log
timeout -k 10 400 python -u tools/ab_vae.py tools/ab/libacehip_head.so > gpurun_out/r04p_ab_vae.log 2>&1 || { tail -20 gpurun_out/r04p_ab_vae.log; exit 1; }
cat gpurun_out/r04p_ab_vae.log
SHAPES=o_half,o timeout -k 10 300 python -u tools/gemm_stamps.py > gpurun_out/r04o_stamps.log 2>&1 || { tail -20 gpurun_out/r04o_stamps.log; exit 1; }
cat gpurun_out/r04o_stamps.log
