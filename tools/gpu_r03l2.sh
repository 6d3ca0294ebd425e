#!/bin/bash
# A/B by swapping the library between runs on one box: head_post weight load ahead of the partials (new) vs HEAD (ref)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_dit.py -k "head or fused or generate" -x -q --timeout 120 --timeout-method thread > gpurun_out/r03l_tests.log 2>&1 || { tail -30 gpurun_out/r03l_tests.log; exit 1; }
tail -1 gpurun_out/r03l_tests.log
for rep in 1 2 3; do for L in new ref; do
cp tools/ab/libacehip_$L.so ace-step-1.5_amd/acehip/libacehip.so
timeout -k 10 300 python bench.py --turbo --seconds 10 --infer-steps 8 --steps 5 --warmup 2 --no-cpu-baseline --no-config1 > gpurun_out/r03l_t.json 2> gpurun_out/r03l_t.err || { tail -20 gpurun_out/r03l_t.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03l_t.json')); print('turbo $L', d['value'], d['dit_ms_per_step'])"
done; done
for L in new ref; do
cp tools/ab/libacehip_$L.so ace-step-1.5_amd/acehip/libacehip.so
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config1 > gpurun_out/r03l_b.json 2> gpurun_out/r03l_b.err || { tail -20 gpurun_out/r03l_b.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03l_b.json')); print('240s $L', d['value'], d['dit_ms_per_step'])"
done
cp tools/ab/libacehip_new.so ace-step-1.5_amd/acehip/libacehip.so
