#!/bin/bash
# Graph vs eager: GPU tests, then the 240 s and turbo 10 s benches with and without the layer-stack graph.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for a in "" "--no-graph" "--turbo --seconds 10 --infer-steps 8 --steps 5 --warmup 2" "--turbo --seconds 10 --infer-steps 8 --steps 5 --warmup 2 --no-graph"; do
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline $a > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "bench failed: $a"; tail -20 gpurun_out/ab.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$a', d['value'], d['dit_ms_per_step'], d['vae_ms_per_song'], d['roofline']['avg_launch_us'])"
done
