#!/bin/bash
# overlapped text encoder: parity, then turbo / 240 s lines with and without the overlap (interleaved)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_condenc.py tests/test_textenc.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r03j_tests.log 2>&1 || { tail -30 gpurun_out/r03j_tests.log; exit 1; }
tail -1 gpurun_out/r03j_tests.log
for rep in 1 2; do
for ov in "" "--no-overlap"; do
timeout -k 10 300 python bench.py --turbo --seconds 10 --infer-steps 8 --steps 5 --warmup 2 --no-cpu-baseline --no-config1 $ov > gpurun_out/r03j_t.json 2> gpurun_out/r03j_t.err || { tail -20 gpurun_out/r03j_t.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03j_t.json')); print('turbo $ov', d['value'], d['dit_ms_per_step'])"
done; done
for ov in "" "--no-overlap"; do
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-config1 $ov > gpurun_out/r03j_b.json 2> gpurun_out/r03j_b.err || { tail -20 gpurun_out/r03j_b.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r03j_b.json')); print('240s $ov', d['value'], d['dit_ms_per_step'])"
done
