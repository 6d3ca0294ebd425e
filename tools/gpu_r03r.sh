#!/bin/bash
# short-song GEMM split sizing / skinny kernel with the folded epilogues; concurrent timbre encoder
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_dit.py -k "splitk or skinny" tests/test_gpu_condenc.py > gpurun_out/r03r_test.log 2>&1 || { tail -30 gpurun_out/r03r_test.log; exit 1; }
tail -1 gpurun_out/r03r_test.log
SONG_SECONDS=10 SONG_TURBO=1 ROUNDS=5 timeout -k 10 300 python -u tools/ab_env_song.py 'ACEHIP_SPLITK_MINK=4' 'ACEHIP_SPLITK_MINK=2' 'ACEHIP_SPLITK_MINK=8' 'ACEHIP_SKINNY=1' 'ACEHIP_SKINNY=1,ACEHIP_SKINNY_D=2' 2>&1 | grep -v amdgpu.ids
for c in 0 1; do ACEHIP_ENC_CONCURRENT=$c timeout -k 10 300 python bench.py --turbo --seconds 10 --infer-steps 8 --steps 5 --warmup 2 --no-cpu-baseline --no-config1 > gpurun_out/r03r_turbo_$c.json 2> gpurun_out/r03r_turbo.err || { tail -20 gpurun_out/r03r_turbo.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03r_turbo_$c.json')); print('concurrent=$c', d['value'], d['dit_ms_per_song'], d['vae_ms_per_song'])"; done
