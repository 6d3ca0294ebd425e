#!/bin/bash
# after the turbo changes: attention + GEMM parity, then the other configs' bench lines
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r03c}
[ "$SKIP_TESTS2" = 1 ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_dit.py tests/test_gpu_sampler.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python bench.py --turbo --seconds 10 --infer-steps 8 --steps 5 --warmup 2 --no-cpu-baseline --no-config1 > gpurun_out/${TAG}_bench_turbo10s.json 2> gpurun_out/${TAG}_turbo.err || { tail -20 gpurun_out/${TAG}_turbo.err; exit 1; }
timeout -k 10 300 python bench.py --seconds 10 --infer-steps 27 --steps 3 --warmup 1 --no-cpu-baseline --no-config1 > gpurun_out/${TAG}_bench_base10s.json 2> gpurun_out/${TAG}_base10.err || { tail -20 gpurun_out/${TAG}_base10.err; exit 1; }
timeout -k 10 400 python bench.py --repaint --steps 2 --warmup 1 --no-cpu-baseline --no-config1 > gpurun_out/${TAG}_bench_repaint.json 2> gpurun_out/${TAG}_repaint.err || { tail -20 gpurun_out/${TAG}_repaint.err; exit 1; }
timeout -k 10 500 python bench.py --seconds 600 --infer-steps 60 --steps 1 --warmup 1 --no-cpu-baseline --no-config1 > gpurun_out/${TAG}_bench_600s.json 2> gpurun_out/${TAG}_600s.err || { tail -20 gpurun_out/${TAG}_600s.err; exit 1; }
for f in turbo10s base10s repaint 600s; do python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_$f.json')); print('$f', d['value'], d['unit'], d.get('dit_ms_per_step'), d.get('vae_ms_per_song'), json.dumps(d.get('kernels')))"; done
