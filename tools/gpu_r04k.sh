#!/bin/bash
# head-post epilogue rewrite: parity tests, one-process A/B against HEAD, store-vs-headpost gap
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fused.py tests/test_gpu_dit.py -k "headpost or golden or forward or qkv" > gpurun_out/r04k_tests.log 2>&1 || { tail -30 gpurun_out/r04k_tests.log; exit 1; }
tail -3 gpurun_out/r04k_tests.log
timeout -k 10 300 python -u tools/ab_headpost.py tools/ab/libacehip_head.so > gpurun_out/r04k_ab_headpost.log 2>&1 || { tail -20 gpurun_out/r04k_ab_headpost.log; exit 1; }
cat gpurun_out/r04k_ab_headpost.log
timeout -k 10 300 python -u tools/bench_headpost.py > gpurun_out/r04k_bench_headpost.log 2>&1 || { tail -20 gpurun_out/r04k_bench_headpost.log; exit 1; }
cat gpurun_out/r04k_bench_headpost.log
