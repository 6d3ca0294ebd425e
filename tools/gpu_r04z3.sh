#!/bin/bash
# end-of-round knob A/Bs at the final tree: HIP-graph replay on the turbo 10 s song, and cross
# attention on attn_pw_kernel (ACEHIP_ATTN_PW 2 → 6) on the 240 s song
set -o pipefail
mkdir -p gpurun_out
SONG_TURBO=1 SONG_SECONDS=10 ROUNDS=5 timeout -k 10 300 python -u tools/ab_env_song.py 'ACEHIP_DIT_GRAPH=0' 'ACEHIP_DIT_GRAPH=1' > gpurun_out/r04z3_ab_graph_turbo.log 2>&1
rc=$?; tail -3 gpurun_out/r04z3_ab_graph_turbo.log; [ $rc -ne 0 ] && exit $rc
ROUNDS=2 timeout -k 10 400 python -u tools/ab_env_song.py 'ACEHIP_ATTN_PW=2' 'ACEHIP_ATTN_PW=6' > gpurun_out/r04z3_ab_pw_cross.log 2>&1
rc=$?; tail -3 gpurun_out/r04z3_ab_pw_cross.log; exit $rc
