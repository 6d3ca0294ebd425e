#!/bin/bash
# attention cost model (per-unit fixed cost vs per-tile cost)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u tools/attn_cost.py > gpurun_out/r03t_attn_cost.jsonl 2> gpurun_out/r03t_attn_cost.err || { tail -20 gpurun_out/r03t_attn_cost.err; exit 1; }
cat gpurun_out/r03t_attn_cost.jsonl
