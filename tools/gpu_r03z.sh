#!/bin/bash
# turbo cross-attention: KV tiles per part of the short split (1 / 2 / 3), in isolation and in the song
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_dit.py -x -q --timeout 120 --timeout-method thread -k "attention" > gpurun_out/r03z_tests.log 2>&1 || { tail -30 gpurun_out/r03z_tests.log; exit 1; }
tail -1 gpurun_out/r03z_tests.log
for t in 2 1 3; do ACEHIP_ATTN_SHORT_TPP=$t ATTN_S=125 ATTN_B=1 SHAPES=cross timeout -k 10 100 python -u tools/bench_attn.py 2>&1 | grep cross | sed "s/^/tpp=$t /"; done
SONG_TURBO=1 SONG_SECONDS=10 timeout -k 10 300 python -u tools/ab_env_song.py 'ACEHIP_ATTN_SHORT_TPP=2' 'ACEHIP_ATTN_SHORT_TPP=1' 'ACEHIP_ATTN_SHORT_TPP=3' > gpurun_out/r03z_ab.log 2>&1 || { tail -20 gpurun_out/r03z_ab.log; exit 1; }
tail -3 gpurun_out/r03z_ab.log
