#!/bin/bash
# conv_out staging / grouped weight loads: VAE parity tests, then the in-process decode A/B
# against HEAD's library and the G = 1 / 2 builds.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_vae.py tests/test_gpu_vae_units.py tests/test_gpu_long.py -m gpu -k "vae or decode or encode" > gpurun_out/r04co_tests.log 2>&1
rc=$?; tail -3 gpurun_out/r04co_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/ab_vae.py tools/ab/libacehip_head.so tools/ab/libacehip_g1.so tools/ab/libacehip_g2.so > gpurun_out/r04co_ab_vae.log 2>&1
rc=$?; cat gpurun_out/r04co_ab_vae.log | tail -3; exit $rc
