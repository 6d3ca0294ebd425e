#!/bin/bash
# Round 4 first GPU pass: the whole -m gpu suite, smoke(), the default bench line.
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r04a}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/${TAG}_gpu_tests.log
[ $rc -ne 0 ] && { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/${TAG}_gpu_tests.log | head -20; exit $rc; }
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
timeout -k 10 300 python -u tools/gemm_stamps.py > gpurun_out/${TAG}_stamps.log 2>&1 || { tail -20 gpurun_out/${TAG}_stamps.log; exit 1; }
cat gpurun_out/${TAG}_stamps.log
VARIANTS=7,8,11 ROUNDS=3 COLD=1 SHAPES=swiglu,down,qkv,o timeout -k 10 300 python -u tools/bench_gemm.py > gpurun_out/${TAG}_bench_gemm.log 2>&1 || { tail -20 gpurun_out/${TAG}_bench_gemm.log; exit 1; }
cat gpurun_out/${TAG}_bench_gemm.log
