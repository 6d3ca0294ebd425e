#!/bin/bash
# attention A/B (working tree vs tools/ab/libacehip_ref.so, one process) + attention parity tests
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_dit.py -k "attention" tests/test_gpu_long.py -k "attention" > gpurun_out/ab_attn_tests.log 2>&1 && \
timeout -k 10 300 python tools/bench_attn.py tools/ab/libacehip_ref.so > gpurun_out/ab_attn.txt 2>&1 && \
ATTN_S=7500 SHAPES=full,band,cross timeout -k 10 300 python tools/bench_attn.py tools/ab/libacehip_ref.so >> gpurun_out/ab_attn.txt 2>&1
