#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
SHAPES=swiglu timeout -k 10 300 python -u tools/bench_small_m.py > gpurun_out/r04t_small_m.log 2>&1 || { tail -20 gpurun_out/r04t_small_m.log; exit 1; }
cat gpurun_out/r04t_small_m.log
M=250 SHAPES=swiglu timeout -k 10 300 python -u tools/bench_small_m.py >> gpurun_out/r04t_small_m.log 2>&1 || { tail -20 gpurun_out/r04t_small_m.log; exit 1; }
tail -1 gpurun_out/r04t_small_m.log
