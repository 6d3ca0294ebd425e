#!/bin/bash
# N = K = 2048 small-M GEMM (O / cross-Q / cross-O at M = 125): split count x tile width
set -o pipefail
mkdir -p gpurun_out
SHAPES=o,qkv,down CASES="m2:ACEHIP_SPLITK_MINK=2;m8:ACEHIP_SPLITK_MINK=8;b64m8:ACEHIP_SPLITK_BN=64+ACEHIP_SPLITK_MINK=8;b64m16:ACEHIP_SPLITK_BN=64+ACEHIP_SPLITK_MINK=16;b128:ACEHIP_SPLITK_BN=128;f2:ACEHIP_SPLITK_FILL=2" timeout -k 10 300 python -u tools/bench_small_m.py > gpurun_out/r03i_small_m.log 2>&1 || { tail -20 gpurun_out/r03i_small_m.log; exit 1; }
cat gpurun_out/r03i_small_m.log
