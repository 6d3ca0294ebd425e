#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for m in 16 64 125 250; do M=$m timeout -k 10 200 python -u tools/bench_skinny.py > gpurun_out/r03e_skinny_$m.log 2>&1 || { tail -30 gpurun_out/r03e_skinny_$m.log; exit 1; }; cat gpurun_out/r03e_skinny_$m.log | grep -v amdgpu.ids; done
