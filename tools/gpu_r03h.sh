#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dit.py -k "streamk or splitk" > gpurun_out/r03h_test.log 2>&1 && \
VARIANTS=7,8,11,14 SHAPES=eq_k6144,eq_k2048,down,qkv,o,swiglu COLD=1 timeout -k 10 300 python -u tools/bench_gemm.py > gpurun_out/r03h_gemm.log 2>&1; rc=$?; tail -3 gpurun_out/r03h_test.log; grep -v amdgpu.ids gpurun_out/r03h_gemm.log; exit $rc
