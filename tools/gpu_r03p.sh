#!/bin/bash
# attention: first K/V tile(s) issued beside the Q loads + 16-B write-through split hand-off
# (tree) vs HEAD's kernels (late build), and the split knobs that the cheaper hand-off may enable
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_dit.py -k "attention" > gpurun_out/r03p_test.log 2>&1 || { tail -30 gpurun_out/r03p_test.log; exit 1; }
tail -1 gpurun_out/r03p_test.log
A="timeout -k 10 200 python -u tools/bench_attn.py tools/ab/libacehip_late.so"
$A 2>&1 | grep -v amdgpu.ids
echo "--- band tail split (PW_SPLIT=4)"; SHAPES=band ACEHIP_ATTN_PW_SPLIT=4 $A 2>&1 | grep -v amdgpu.ids
for n in 2 3 4; do echo "--- cross1 split-all $n"; SHAPES=cross1 ACEHIP_ATTN_SPLIT_ALL=$n $A 2>&1 | grep -v amdgpu.ids; done
echo "--- turbo S=125"; ATTN_S=125 ATTN_B=1 $A 2>&1 | grep -v amdgpu.ids
echo "--- turbo S=125 TPP=1"; ACEHIP_ATTN_SHORT_TPP=1 ATTN_S=125 ATTN_B=1 $A 2>&1 | grep -v amdgpu.ids
