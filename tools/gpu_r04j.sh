#!/bin/bash
# kernel trace of one bench song at HEAD: per-kernel stats + where the blit copies come from
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rm -rf gpurun_out/kt
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/kt -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/r04j_bench.json 2> gpurun_out/r04j.err || { tail -20 gpurun_out/r04j.err; exit 1; }
DB=$(find gpurun_out/kt -name "*.db" | head -1)
python3 tools/diag_copies.py $DB > gpurun_out/r04j_copies.txt 2>&1
python3 tools/rocprof_summary.py $DB > gpurun_out/r04j_kernel_stats.md 2>&1
rm -rf gpurun_out/kt
cat gpurun_out/r04j_copies.txt
head -40 gpurun_out/r04j_kernel_stats.md
