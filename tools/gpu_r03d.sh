#!/bin/bash
set -o pipefail
mkdir -p gpurun_out

timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu "tests/test_gpu_dit.py::test_gemm_splitk_small_m" "tests/test_gpu_dit.py::test_apg_euler_multichunk" "tests/test_gpu_dit.py::test_apg_euler_kernel_replay" tests/test_gpu_sampler.py tests/test_gpu_fused.py > gpurun_out/r03d_small.log 2>&1; rc=$?; tail -15 gpurun_out/r03d_small.log; [ $rc = 0 ] || exit 1
timeout -k 10 200 python -u tools/bench_skinny.py > gpurun_out/r03d_skinny.log 2>&1 || { tail -30 gpurun_out/r03d_skinny.log; exit 1; }
cat gpurun_out/r03d_skinny.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --seconds 10 --infer-steps 8 --turbo > gpurun_out/r03d_turbo.json 2> gpurun_out/r03d_turbo.err || { tail -30 gpurun_out/r03d_turbo.err; exit 1; }
cat gpurun_out/r03d_turbo.json
