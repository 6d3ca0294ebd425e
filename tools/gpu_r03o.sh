#!/bin/bash
# encoder split-K epilogue deferral: tests, then the turbo 10 s bench line (encoders inside)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_textenc.py tests/test_gpu_condenc.py tests/test_gpu_fused.py > gpurun_out/r03o_test.log 2>&1 || { tail -30 gpurun_out/r03o_test.log; exit 1; }
tail -2 gpurun_out/r03o_test.log
timeout -k 10 300 python bench.py --turbo --seconds 10 --infer-steps 8 --steps 5 --warmup 2 --no-cpu-baseline --no-config1 > gpurun_out/r03o_turbo.json 2> gpurun_out/r03o_turbo.err || { tail -20 gpurun_out/r03o_turbo.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03o_turbo.json')); print(d['value'], d['dit_ms_per_song'], d['vae_ms_per_song'], d['kernels'])"
