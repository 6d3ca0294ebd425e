#!/bin/bash
# small-M defaults: GEMM parity, turbo song A/B (whole-K SwiGLU, split-K BN 64) and bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dit.py -x -q --timeout 120 --timeout-method thread -k "gemm or generate" > gpurun_out/r03y_tests.log 2>&1 || { tail -30 gpurun_out/r03y_tests.log; exit 1; }
tail -2 gpurun_out/r03y_tests.log
SONG_TURBO=1 SONG_SECONDS=10 timeout -k 10 300 python -u tools/ab_env_song.py 'ACEHIP_SMALLM_WHOLEK=1' 'ACEHIP_SMALLM_WHOLEK=0,ACEHIP_SPLITK_BN=128' 'ACEHIP_SMALLM_WHOLEK=0' 'ACEHIP_SPLITK_BN=128' > gpurun_out/r03y_ab_turbo.log 2>&1 || { tail -20 gpurun_out/r03y_ab_turbo.log; exit 1; }
tail -5 gpurun_out/r03y_ab_turbo.log
timeout -k 10 300 python bench.py --turbo --seconds 10 --infer-steps 8 --steps 5 --warmup 2 --no-cpu-baseline --no-config1 > gpurun_out/r03y_bench_turbo10s.json 2> gpurun_out/r03y_turbo.err || { tail -20 gpurun_out/r03y_turbo.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03y_bench_turbo10s.json')); print(d['value'], d['dit_ms_per_step'], d['vae_ms_per_song'], json.dumps(d['kernels']))"
