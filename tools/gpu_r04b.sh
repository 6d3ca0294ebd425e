#!/bin/bash
# GEMM epilogue VALU cuts: suite, in-process A/B vs the HEAD library, stamps, bench line
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r04b}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_gpu_tests.log
[ $rc -ne 0 ] && { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/${TAG}_gpu_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/ab_gemm.py tools/ab/libacehip_head.so > gpurun_out/${TAG}_ab_gemm.log 2>&1 || { tail -20 gpurun_out/${TAG}_ab_gemm.log; exit 1; }
cat gpurun_out/${TAG}_ab_gemm.log
SHAPES=swiglu,down,o timeout -k 10 300 python -u tools/gemm_stamps.py > gpurun_out/${TAG}_stamps.log 2>&1 || { tail -20 gpurun_out/${TAG}_stamps.log; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
