#!/bin/bash
# One GPU-box session: GPU tests, bench (with CPU baseline), rocprof kernel trace of the bench,
# then separate PMC passes (FETCH_SIZE, WRITE_SIZE; kernel-trace only) on tools/prof_dit.py.
set -o pipefail
mkdir -p gpurun_out
lscpu | grep -E "Model name|^CPU\(s\)" > gpurun_out/host.txt
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
echo "pytest rc=$?"; tail -4 gpurun_out/gpu_tests.log
[ "$SKIP_BENCH" = 1 ] && exit 0
timeout -k 10 900 python bench.py --steps 2 --warmup 1 $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rm -rf gpurun_out/prof gpurun_out/pmc_fetch gpurun_out/pmc_write
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof_bench.json 2> gpurun_out/prof.err || { echo "rocprof failed"; tail -20 gpurun_out/prof.err; exit 1; }
[ "$SKIP_PMC" = 1 ] && exit 0
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run -- python3 tools/prof_dit.py --forwards 1 --vae > gpurun_out/pmc1.log 2>&1 || { tail -20 gpurun_out/pmc1.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run -- python3 tools/prof_dit.py --forwards 1 --vae > gpurun_out/pmc2.log 2>&1 || { tail -20 gpurun_out/pmc2.log; exit 1; }
echo "pmc ok"
