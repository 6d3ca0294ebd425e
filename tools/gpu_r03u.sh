#!/bin/bash
# persistent band attention: parity tests, then the band cost points
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_dit.py -x -q --timeout 120 --timeout-method thread -k "attention" > gpurun_out/r03u_tests.log 2>&1 || { tail -30 gpurun_out/r03u_tests.log; exit 1; }
tail -3 gpurun_out/r03u_tests.log
BAND_ONLY=1 timeout -k 10 200 python -u tools/attn_cost.py > gpurun_out/r03u_attn_cost.jsonl 2> gpurun_out/r03u_attn_cost.err || { tail -20 gpurun_out/r03u_attn_cost.err; exit 1; }
cat gpurun_out/r03u_attn_cost.jsonl
# turbo 10 s song: bench line + kernel-trace stats
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python bench.py --turbo --seconds 10 --infer-steps 8 --steps 5 --warmup 2 --no-cpu-baseline --no-config1 > gpurun_out/r03u_bench_turbo10s.json 2> gpurun_out/r03u_turbo.err || { tail -20 gpurun_out/r03u_turbo.err; exit 1; }
rm -rf gpurun_out/proft
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/proft -o run -- python3 bench.py --turbo --seconds 10 --infer-steps 8 --steps 3 --warmup 1 --no-cpu-baseline --no-config1 > gpurun_out/r03u_prof_turbo.json 2> gpurun_out/r03u_proft.err || { tail -20 gpurun_out/r03u_proft.err; exit 1; }
python3 tools/rocprof_summary.py $(find gpurun_out/proft -name "*.db" | head -1) > gpurun_out/r03u_turbo10s_kernel_stats.md
rm -rf gpurun_out/proft
python3 -c "import json; d=json.load(open('gpurun_out/r03u_bench_turbo10s.json')); print(d['value'], d['dit_ms_per_step'], d['vae_ms_per_song'], json.dumps(d['kernels']))"
head -40 gpurun_out/r03u_turbo10s_kernel_stats.md
