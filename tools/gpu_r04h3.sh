#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
SONG_TURBO=1 SONG_SECONDS=10 ROUNDS=6 timeout -k 10 400 python -u tools/ab_env_song.py 'ACEHIP_SPLITK_BN=0' 'ACEHIP_SPLITK_BN=64' 'ACEHIP_SMALLM_WHOLEK=2' 'ACEHIP_SPLITK_BN=64,ACEHIP_SMALLM_WHOLEK=2' > gpurun_out/r04h3_ab_turbo.log 2>&1 || { tail -20 gpurun_out/r04h3_ab_turbo.log; exit 1; }
cat gpurun_out/r04h3_ab_turbo.log
SONG_SECONDS=10 ROUNDS=4 timeout -k 10 400 python -u tools/ab_env_song.py 'ACEHIP_SPLITK_BN=0' 'ACEHIP_SPLITK_BN=64' 'ACEHIP_SMALLM_WHOLEK=2' > gpurun_out/r04h3_ab_base10.log 2>&1 || { tail -20 gpurun_out/r04h3_ab_base10.log; exit 1; }
cat gpurun_out/r04h3_ab_base10.log
