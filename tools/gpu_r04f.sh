#!/bin/bash
# dual-stream null-row MLP: parity at full length, then the song A/B
set -o pipefail
mkdir -p gpurun_out
ACEHIP_DIT_DUAL=1 timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_long.py -k "cfg" > gpurun_out/r04f_long_dual.log 2>&1 || { tail -30 gpurun_out/r04f_long_dual.log; exit 1; }
tail -6 gpurun_out/r04f_long_dual.log
ROUNDS=4 timeout -k 10 400 python -u tools/ab_env_song.py 'ACEHIP_DIT_DUAL=0' 'ACEHIP_DIT_DUAL=1' > gpurun_out/r04f_ab_dual.log 2>&1 || { tail -20 gpurun_out/r04f_ab_dual.log; exit 1; }
cat gpurun_out/r04f_ab_dual.log
# SQ pass over one 240 s VAE decode: where the residual-unit kernels wait
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"
rm -rf gpurun_out/pv
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace -d gpurun_out/pv -o run -- python3 tools/prof_dit.py --forwards 0 --vae > gpurun_out/r04f_pv.log 2>&1 || { tail -5 gpurun_out/r04f_pv.log; exit 1; }
python3 tools/pmc_sq.py $(find gpurun_out/pv -name "*.db" | head -1) gpurun_out/r04f_pmc_vae_sq.json
rm -rf gpurun_out/pv
