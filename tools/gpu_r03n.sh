#!/bin/bash
# weight prefetch for short songs: turbo 10 s DiT song, prefetch off / on at several widths
set -o pipefail
mkdir -p gpurun_out
SONG_SECONDS=10 SONG_TURBO=1 ROUNDS=7 timeout -k 10 300 python -u tools/ab_env_song.py 'ACEHIP_PREFETCH=0' 'ACEHIP_PREFETCH=1,ACEHIP_PREFETCH_BLOCKS=8' 'ACEHIP_PREFETCH=1,ACEHIP_PREFETCH_BLOCKS=24' 'ACEHIP_PREFETCH=1,ACEHIP_PREFETCH_BLOCKS=64' 2>&1 | grep -v amdgpu.ids
