#!/bin/bash
# GPU tests + default bench (no CPU baseline) + rocprof kernel trace of the bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -30 gpurun_out/bench.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench.json')); print(d['value'], d['dit_ms_per_step'], d['dit_ms_per_song'], d['vae_ms_per_song'], d['roofline']['achieved'], d['config']['workload'])"
