#!/bin/bash
# per-wave band ranges (ACEHIP_ATTN_SHIFT=1): parity, band A/B in isolation, 240 s song A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_gpu_dit.py -x -v --timeout 120 --timeout-method thread -k "band_shift or band_persistent or attention_tail" > gpurun_out/r03n2_tests.log 2>&1 || { tail -30 gpurun_out/r03n2_tests.log; exit 1; }
tail -2 gpurun_out/r03n2_tests.log
for S in 3000 6000; do ATTN_S=$S SHAPES=band timeout -k 10 120 python -u tools/ab_env_attn.py '' 'ACEHIP_ATTN_PERSIST=0' 'ACEHIP_ATTN_SHIFT=1' 2>&1 | sed "s/^/S=$S /" || exit 1; done
SONG_SECONDS=240 timeout -k 10 400 python -u tools/ab_env_song.py '' 'ACEHIP_ATTN_SHIFT=1' > gpurun_out/r03n2_ab.log 2>&1 || { tail -20 gpurun_out/r03n2_ab.log; exit 1; }
tail -3 gpurun_out/r03n2_ab.log
