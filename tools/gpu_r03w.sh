#!/bin/bash
# cheaper split hand-off (16-B sc1 slabs, last arriver keeps its own part): parity + A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dit.py -x -q --timeout 120 --timeout-method thread -k "attention" > gpurun_out/r03w_tests.log 2>&1 || { tail -30 gpurun_out/r03w_tests.log; exit 1; }
tail -2 gpurun_out/r03w_tests.log
SHAPES=full,band,cross,cross1 timeout -k 10 200 python -u tools/bench_attn.py tools/ab/libacehip_ref.so > gpurun_out/r03w_attn_ab.log 2>&1 || { tail -20 gpurun_out/r03w_attn_ab.log; exit 1; }
cat gpurun_out/r03w_attn_ab.log
ATTN_S=125 ATTN_B=1 SHAPES=full,band,cross timeout -k 10 200 python -u tools/bench_attn.py tools/ab/libacehip_ref.so > gpurun_out/r03w_attn_ab125.log 2>&1 || { tail -20 gpurun_out/r03w_attn_ab125.log; exit 1; }
cat gpurun_out/r03w_attn_ab125.log
