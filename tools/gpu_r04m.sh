#!/bin/bash
# rmsnorm VALU cut: parity tests, one-process A/B against HEAD
set -o pipefail
mkdir -p gpurun_out
#timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_fused.py tests/test_gpu_dit.py -k "rmsnorm or norm or golden or forward" > gpurun_out/r04m_tests.log 2>&1 || { tail -30 gpurun_out/r04m_tests.log; exit 1; }
#tail -3
RPW=2,4,-2,-4 timeout -k 10 300 python -u tools/ab_norm.py tools/ab/libacehip_head.so > gpurun_out/r04m_ab_norm.log 2>&1 || { tail -20 gpurun_out/r04m_ab_norm.log; exit 1; }
cat gpurun_out/r04m_ab_norm.log
