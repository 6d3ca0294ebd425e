#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/attn_full_cost.py > gpurun_out/r03v_attn_full.jsonl 2> gpurun_out/r03v_attn_full.err || { tail -20 gpurun_out/r03v_attn_full.err; exit 1; }
cat gpurun_out/r03v_attn_full.jsonl
# DiT song A/B: full attention on attn_pw_kernel (mask 3) vs attn_fwd_kernel (mask 2, default)
timeout -k 10 400 python -u tools/ab_env_song.py 'ACEHIP_ATTN_PW=2' 'ACEHIP_ATTN_PW=3' > gpurun_out/r03v_ab_pw.log 2>&1 || { tail -20 gpurun_out/r03v_ab_pw.log; exit 1; }
tail -8 gpurun_out/r03v_ab_pw.log
