#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
VARIANTS=7,8,11 SHAPES=down,qkv,o,swiglu COLD=1 timeout -k 10 300 python -u tools/bench_gemm.py > gpurun_out/r03f_gemm.log 2>&1; cat gpurun_out/r03f_gemm.log | grep -v amdgpu.ids
