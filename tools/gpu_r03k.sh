#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dit.py -k "gemm" > gpurun_out/r03k_test.log 2>&1 || { tail -20 gpurun_out/r03k_test.log; exit 1; }
tail -1 gpurun_out/r03k_test.log
for c in 0 1; do
echo "COLD=$c"
ROUNDS=3 VARIANTS=11,30,29,8,7 SHAPES=down,qkv COLD=$c timeout -k 10 300 python -u tools/bench_gemm.py > gpurun_out/r03k_gemm.log 2>&1 || exit 1; grep -v amdgpu.ids gpurun_out/r03k_gemm.log
done
