#!/bin/bash
# hipBLASLt for the N <= 4096 projections (ACEHIP_BLASLT bit mask): DiT parity with it on, 240 s song A/B
set -o pipefail
mkdir -p gpurun_out
[ -n "$SKIP1" ] || ACEHIP_BLASLT=7 timeout -k 10 400 python -u -m pytest tests/test_gpu_dit.py tests/test_gpu_long.py -x -q -k "not blaslt" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r03n5_tests.log 2>&1 || { tail -40 gpurun_out/r03n5_tests.log; exit 1; }
[ -n "$SKIP1" ] || tail -2 gpurun_out/r03n5_tests.log
timeout -k 10 200 python -u -m pytest tests/test_gpu_dit.py -x -q --timeout 150 --timeout-method thread -p no:cacheprovider -k blaslt > gpurun_out/r03n5_t2.log 2>&1 || { tail -30 gpurun_out/r03n5_t2.log; exit 1; }
tail -1 gpurun_out/r03n5_t2.log
SONG_SECONDS=240 timeout -k 10 500 python -u tools/ab_env_song.py '' 'ACEHIP_BLASLT=1' 'ACEHIP_BLASLT=2' 'ACEHIP_BLASLT=4' 'ACEHIP_BLASLT=7' > gpurun_out/r03n5_ab.log 2>&1 || { tail -20 gpurun_out/r03n5_ab.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r03n5_ab.log | tail -6
