#!/bin/bash
# split-K ring depth / split count at the turbo shapes (M = 125)
set -o pipefail
mkdir -p gpurun_out
CASES="st4:ACEHIP_SPLITK_STAGES=4;st6:ACEHIP_SPLITK_STAGES=6;k2:ACEHIP_SPLITK_KMIN=2;k2st6:ACEHIP_SPLITK_KMIN=2+ACEHIP_SPLITK_STAGES=6;k8:ACEHIP_SPLITK_KMIN=8+ACEHIP_SPLITK_STAGES=6;k2bn64:ACEHIP_SPLITK_KMIN=2+ACEHIP_SPLITK_BN=64+ACEHIP_SPLITK_STAGES=6" SHAPES=down,qkv,o timeout -k 10 400 python -u tools/bench_small_m.py > gpurun_out/r04l_small_m.log 2>&1 || { tail -20 gpurun_out/r04l_small_m.log; exit 1; }
cat gpurun_out/r04l_small_m.log
