#!/bin/bash
# ru8_kernel (256-row residual-unit tiles, DMA helper waves, 3-slot W ring): unit parity vs
# torch and bit-equality with ru7, then the 240 s decode A/B (ACEHIP_RU7 = 1 vs 2).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_vae_units.py -k resunit > gpurun_out/r04ru8_tests.log 2>&1
rc=$?; tail -15 gpurun_out/r04ru8_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/ab_env_vae.py 'ACEHIP_RU7=1' 'ACEHIP_RU7=2' > gpurun_out/r04ru8_ab_vae.log 2>&1
rc=$?; tail -5 gpurun_out/r04ru8_ab_vae.log; exit $rc
