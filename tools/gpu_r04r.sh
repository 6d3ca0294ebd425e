#!/bin/bash
# helper-wave four-wave tile as production variant 13: suite, A/B against HEAD, bench
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r04r}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_gpu_tests.log
[ $rc -ne 0 ] && { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/${TAG}_gpu_tests.log | head -20; exit $rc; }
SHAPES=o_half,crossq timeout -k 10 300 python -u tools/ab_gemm.py tools/ab/libacehip_head.so > gpurun_out/${TAG}_ab_gemm.log 2>&1 || { tail -20 gpurun_out/${TAG}_ab_gemm.log; exit 1; }
cat gpurun_out/${TAG}_ab_gemm.log
timeout -k 10 300 python -u tools/ab_headpost.py tools/ab/libacehip_head.so > gpurun_out/${TAG}_ab_headpost.log 2>&1 || { tail -20 gpurun_out/${TAG}_ab_headpost.log; exit 1; }
cat gpurun_out/${TAG}_ab_headpost.log
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
