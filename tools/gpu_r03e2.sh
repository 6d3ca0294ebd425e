#!/bin/bash
# launch-attached SwiGLU events: parity + profile tests, turbo / 240 s bench lines, turbo timeline
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python -u -m pytest tests/test_gpu_dit.py tests/test_gpu_integration.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r03e_tests.log 2>&1 || { tail -30 gpurun_out/r03e_tests.log; exit 1; }
tail -1 gpurun_out/r03e_tests.log
timeout -k 10 300 python bench.py --turbo --seconds 10 --infer-steps 8 --steps 5 --warmup 2 --no-cpu-baseline --no-config1 > gpurun_out/r03e_bench_turbo10s.json 2> gpurun_out/r03e_turbo.err || { tail -20 gpurun_out/r03e_turbo.err; exit 1; }
timeout -k 10 400 python bench.py --no-cpu-baseline --no-config1 > gpurun_out/r03e_bench.json 2> gpurun_out/r03e_bench.err || { tail -20 gpurun_out/r03e_bench.err; exit 1; }
for f in bench_turbo10s bench; do python3 -c "import json; d=json.load(open('gpurun_out/r03e_$f.json')); r=d['roofline']; print('$f', d['value'], d['dit_ms_per_step'], d['vae_ms_per_song'], r['avg_launch_us'], r['launches'], r['frac'], d['kernels']['gemm_swiglu'])"; done
rm -rf gpurun_out/tl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tl -o run -- python3 bench.py --turbo --seconds 10 --infer-steps 8 --steps 1 --warmup 1 --no-cpu-baseline --no-config1 > gpurun_out/r03e_tl_bench.json 2> gpurun_out/r03e_tl.err || { tail -20 gpurun_out/r03e_tl.err; exit 1; }
DB=$(find gpurun_out/tl -name "*.db" | head -1)
python3 tools/timeline.py $DB --mark wav_peak --nth 1 --count 3600 > gpurun_out/r03e_timeline.txt
python3 tools/rocprof_summary.py $DB > gpurun_out/r03e_turbo_kernel_stats.md
rm -rf gpurun_out/tl
grep "window" gpurun_out/r03e_timeline.txt
grep -m3 "grid=49152x1$" -B1 -A1 gpurun_out/r03e_timeline.txt | cut -c1-120
