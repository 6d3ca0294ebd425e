#!/bin/bash
# Re-entry check of the restored tree: the whole -m gpu suite, then the turbo 10 s line
# and its kernel-trace stats (where the short-song time goes).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03l_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r03l_gpu_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --turbo --seconds 10 --infer-steps 8 --steps 5 --warmup 2 --no-cpu-baseline --no-config1 > gpurun_out/r03l_turbo.json 2> gpurun_out/r03l_turbo.err || { tail -20 gpurun_out/r03l_turbo.err; exit 1; }
cat gpurun_out/r03l_turbo.json
rm -rf gpurun_out/kt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt -o run -- python3 bench.py --turbo --seconds 10 --infer-steps 8 --steps 3 --warmup 1 --no-cpu-baseline --no-config1 > gpurun_out/r03l_turbo_prof.json 2> gpurun_out/r03l_prof.err || { tail -20 gpurun_out/r03l_prof.err; exit 1; }
NAMEW=200 python3 tools/rocprof_summary.py $(find gpurun_out/kt -name "*.db" | head -1) > gpurun_out/r03l_turbo_stats.md
rc=$?
rm -rf gpurun_out/kt
exit $rc
