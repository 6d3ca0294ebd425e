#!/bin/bash
# timestep GEMVs (silu once, W prefetch): timestep / schedule parity tests, turbo line, GEMV timing
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest tests/test_gpu_dit.py tests/test_gpu_sampler.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03h_tests.log 2>&1 || { tail -30 gpurun_out/r03h_tests.log; exit 1; }
tail -1 gpurun_out/r03h_tests.log
timeout -k 10 300 python bench.py --turbo --seconds 10 --infer-steps 8 --steps 5 --warmup 2 --no-cpu-baseline --no-config1 > gpurun_out/r03h_bench_turbo10s.json 2> gpurun_out/r03h_turbo.err || { tail -20 gpurun_out/r03h_turbo.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03h_bench_turbo10s.json')); print(d['value'], d['dit_ms_per_step'], d['vae_ms_per_song'])"
rm -rf gpurun_out/tl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tl -o run -- python3 bench.py --turbo --seconds 10 --infer-steps 8 --steps 1 --warmup 1 --no-cpu-baseline --no-config1 > gpurun_out/r03h_tl_bench.json 2> gpurun_out/r03h_tl.err || { tail -20 gpurun_out/r03h_tl.err; exit 1; }
DB=$(find gpurun_out/tl -name "*.db" | head -1)
python3 tools/rocprof_summary.py $DB > gpurun_out/r03h_turbo_kernel_stats.md
rm -rf gpurun_out/tl
grep -E "gemv|silu" gpurun_out/r03h_turbo_kernel_stats.md
