#!/bin/bash
# batched cross K/V projections: DiT / sampler / integration / encoder parity, turbo + 240 s lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_dit.py tests/test_gpu_sampler.py tests/test_gpu_integration.py tests/test_gpu_fp32.py tests/test_gpu_condenc.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03f_tests.log 2>&1 || { tail -30 gpurun_out/r03f_tests.log; exit 1; }
tail -1 gpurun_out/r03f_tests.log
timeout -k 10 300 python bench.py --turbo --seconds 10 --infer-steps 8 --steps 5 --warmup 2 --no-cpu-baseline --no-config1 > gpurun_out/r03f_bench_turbo10s.json 2> gpurun_out/r03f_turbo.err || { tail -20 gpurun_out/r03f_turbo.err; exit 1; }
timeout -k 10 400 python bench.py --no-cpu-baseline --no-config1 > gpurun_out/r03f_bench.json 2> gpurun_out/r03f_bench.err || { tail -20 gpurun_out/r03f_bench.err; exit 1; }
for f in bench_turbo10s bench; do python3 -c "import json; d=json.load(open('gpurun_out/r03f_$f.json')); r=d['roofline']; print('$f', d['value'], d['dit_ms_per_step'], d['vae_ms_per_song'], r['avg_launch_us'], r['frac'])"; done
