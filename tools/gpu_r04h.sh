#!/bin/bash
# two-phase ping-pong schedule as production: suite, song A/B against the four-phase arm, bench
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r04h}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_gpu_tests.log
[ $rc -ne 0 ] && { grep -E "^(FAILED|ERROR)|Error|assert" gpurun_out/${TAG}_gpu_tests.log | head -20; exit $rc; }
ROUNDS=3 timeout -k 10 400 python -u tools/ab_env_song.py 'ACEHIP_GEMM_PPSCHED=1' 'ACEHIP_GEMM_PPSCHED=2' > gpurun_out/${TAG}_ab_song.log 2>&1 || { tail -20 gpurun_out/${TAG}_ab_song.log; exit 1; }
cat gpurun_out/${TAG}_ab_song.log
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
