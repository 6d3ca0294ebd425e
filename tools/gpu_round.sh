#!/bin/bash
# One GPU-box session: GPU tests, bench (with CPU baseline), rocprof kernel-trace summary.
set -o pipefail
mkdir -p gpurun_out
lscpu | grep -E "Model name|^CPU\(s\)" > gpurun_out/host.txt
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
echo "pytest rc=$?"; tail -5 gpurun_out/gpu_tests.log
timeout -k 10 900 python bench.py --steps 2 --warmup 1 > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err || { echo "rocprof failed"; tail -20 gpurun_out/prof.err; exit 1; }
find gpurun_out/prof -name "*stats*" | head
