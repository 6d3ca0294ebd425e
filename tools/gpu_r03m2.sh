#!/bin/bash
# turbo cross-attention parts: 3 / 4 / 6 tiles per part, in the song
set -o pipefail
mkdir -p gpurun_out
for t in 3 4 6; do ACEHIP_ATTN_SHORT_TPP=$t ATTN_S=125 ATTN_B=1 SHAPES=cross timeout -k 10 100 python -u tools/bench_attn.py 2>&1 | grep cross | sed "s/^/tpp=$t /"; done
SONG_TURBO=1 SONG_SECONDS=10 timeout -k 10 300 python -u tools/ab_env_song.py 'ACEHIP_ATTN_SHORT_TPP=3' 'ACEHIP_ATTN_SHORT_TPP=4' 'ACEHIP_ATTN_SHORT_TPP=6' > gpurun_out/r03m_ab.log 2>&1 || { tail -20 gpurun_out/r03m_ab.log; exit 1; }
tail -3 gpurun_out/r03m_ab.log
