#!/bin/bash
# clock stamps of the two-phase ping-pong tiles
set -o pipefail
mkdir -p gpurun_out
SHAPES=o_half,o timeout -k 10 300 python -u tools/gemm_stamps.py > gpurun_out/r04o_stamps.log 2>&1 || { tail -20 gpurun_out/r04o_stamps.log; exit 1; }
cat gpurun_out/r04o_stamps.log
