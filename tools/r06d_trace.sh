#!/bin/bash
# one kernel trace of the bench song: per-kernel table, where the blit copies come from, idle gaps
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r06d_tr -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-output-leg > gpurun_out/r06d_bench.log 2>&1 || exit $?
db=$(find gpurun_out/r06d_tr -name "*.db" | head -1)
python3 tools/diag_copies.py $db > gpurun_out/r06d_copies.txt 2>&1
python3 tools/rocprof_summary.py $db > gpurun_out/r06d_kernel_stats.md
rm -rf gpurun_out/r06d_tr
timeout -k 10 600 python3 tools/trace_gaps.py r06d > gpurun_out/r06d_gaps.txt 2>&1
