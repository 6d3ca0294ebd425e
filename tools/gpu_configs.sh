#!/bin/bash
# The other BASELINE configs on one box: 600 s / 60 steps (config 4), repaint (config 5), turbo 10 s (config 0 shape on the GPU).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --seconds 600 --infer-steps 60 > gpurun_out/bench_600s.json 2> gpurun_out/b600.err || { tail -20 gpurun_out/b600.err; exit 1; }
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --repaint > gpurun_out/bench_repaint.json 2> gpurun_out/brp.err || { tail -20 gpurun_out/brp.err; exit 1; }
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --turbo --seconds 10 --infer-steps 8 > gpurun_out/bench_turbo10s.json 2> gpurun_out/btu.err || { tail -20 gpurun_out/btu.err; exit 1; }
for f in 600s repaint turbo10s; do python -c "import json; d=json.load(open('gpurun_out/bench_$f.json')); print('$f', d['value'], d['dit_ms_per_step'], d['vae_ms_per_song'], d['roofline']['achieved'])"; done
