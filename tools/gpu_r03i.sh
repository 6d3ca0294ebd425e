#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rm -rf gpurun_out/kt
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/kt -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r03i_bench.json 2> gpurun_out/r03i.err || { tail -20 gpurun_out/r03i.err; exit 1; }
python3 tools/diag_copies.py $(find gpurun_out/kt -name "*.db" | head -1) > gpurun_out/r03i_copies.txt 2>&1; rc=$?
cat gpurun_out/r03i_copies.txt
rm -rf gpurun_out/kt
exit $rc
