#!/bin/bash
# helper waves in the small-M tiles (variant 17, split-K with ACEHIP_GEMM_SKHELP=1) — historical: the split-K helper switch was removed after this A/B (no gain)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dit.py -k "gemm_variants or small" > gpurun_out/r04h2_tests.log 2>&1 || { tail -30 gpurun_out/r04h2_tests.log; exit 1; }
ACEHIP_GEMM_SKHELP=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dit.py -k "small or splitk" >> gpurun_out/r04h2_tests.log 2>&1 || { tail -30 gpurun_out/r04h2_tests.log; exit 1; }
grep -E "passed|failed" gpurun_out/r04h2_tests.log
timeout -k 10 300 python -u tools/bench_small_m.py > gpurun_out/r04h2_small_m.log 2>&1 || { tail -20 gpurun_out/r04h2_small_m.log; exit 1; }
cat gpurun_out/r04h2_small_m.log
SONG_TURBO=1 SONG_SECONDS=10 ROUNDS=5 timeout -k 10 300 python -u tools/ab_env_song.py 'ACEHIP_GEMM_SKHELP=0' 'ACEHIP_GEMM_SKHELP=1' > gpurun_out/r04h2_ab_turbo.log 2>&1 || { tail -20 gpurun_out/r04h2_ab_turbo.log; exit 1; }
cat gpurun_out/r04h2_ab_turbo.log
