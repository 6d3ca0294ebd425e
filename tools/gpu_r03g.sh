#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu "tests/test_gpu_dit.py::test_gemm_streamk" > gpurun_out/r03g_sk.log 2>&1; rc=$?; grep -E "PASS|FAIL|SKIP|Error|assert" gpurun_out/r03g_sk.log | head -30; [ $rc = 0 ] || exit 1
VARIANTS=8,11,14 SHAPES=down,qkv,o,swiglu COLD=1 timeout -k 10 300 python -u tools/bench_gemm.py > gpurun_out/r03g_gemm.log 2>&1; grep -v amdgpu.ids gpurun_out/r03g_gemm.log
timeout -k 10 600 python -u tools/ab_env_song.py 'ACEHIP_GEMM_SK=0' 'ACEHIP_GEMM_SK=1' > gpurun_out/r03g_song.log 2>&1; tail -8 gpurun_out/r03g_song.log
