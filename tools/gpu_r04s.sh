#!/bin/bash
# conv7 helper waves: VAE parity with them on, decode A/B
set -o pipefail
mkdir -p gpurun_out
ACEHIP_CONV7_NH=2 timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_vae_units.py tests/test_vae.py tests/test_gpu_long.py -m gpu -k "vae or decode or conv" > gpurun_out/r04s_tests.log 2>&1 || { tail -30 gpurun_out/r04s_tests.log; exit 1; }
tail -2 gpurun_out/r04s_tests.log
ROUNDS=5 timeout -k 10 400 python -u tools/ab_env_vae.py 'ACEHIP_CONV7_NH=0' 'ACEHIP_CONV7_NH=2' > gpurun_out/r04s_ab_vae.log 2>&1 || { tail -20 gpurun_out/r04s_ab_vae.log; exit 1; }
cat gpurun_out/r04s_ab_vae.log
