#!/bin/bash
# split-K epilogue fusion: its parity tests, the short-song GEMM tests, then the turbo 10 s and
# a base 10 s (CFG, M = 250) DiT song with the fusion on / off, interleaved in one process
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_dit.py -k "splitk or null_row or production or dedup or turbo or forward_step or golden" tests/test_gpu_fused.py > gpurun_out/r03m_test.log 2>&1 || { tail -30 gpurun_out/r03m_test.log; exit 1; }
tail -2 gpurun_out/r03m_test.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_condenc.py tests/test_textenc.py > gpurun_out/r03m_test2.log 2>&1 || { tail -30 gpurun_out/r03m_test2.log; exit 1; }
tail -2 gpurun_out/r03m_test2.log
SONG_SECONDS=10 SONG_TURBO=1 ROUNDS=7 timeout -k 10 300 python -u tools/ab_env_song.py 'ACEHIP_SPLITK_FUSE=0' 'ACEHIP_SPLITK_FUSE=1' 2>&1 | grep -v amdgpu.ids
SONG_SECONDS=10 ROUNDS=5 timeout -k 10 300 python -u tools/ab_env_song.py 'ACEHIP_SPLITK_FUSE=0' 'ACEHIP_SPLITK_FUSE=1' 2>&1 | grep -v amdgpu.ids
