#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
A="timeout -k 10 200 python -u tools/bench_attn.py tools/ab/libacehip_pwlate.so tools/ab/libacehip_late.so"
timeout -k 10 100 python -u tools/diag_split.py 2>&1 | grep -v amdgpu.ids | head -3
$A 2>&1 | grep -v amdgpu.ids
SHAPES=full,band ATTN_S=125 ATTN_B=1 $A 2>&1 | grep -v amdgpu.ids
