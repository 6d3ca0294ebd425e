#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 120 python -u tools/diag_apg.py > gpurun_out/r03b_diag.log 2>&1; cat gpurun_out/r03b_diag.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu "tests/test_gpu_dit.py::test_gemm_splitk_small_m" tests/test_gpu_fused.py > gpurun_out/r03b_small.log 2>&1 || { tail -30 gpurun_out/r03b_small.log; exit 1; }
tail -2 gpurun_out/r03b_small.log
timeout -k 10 200 python -u tools/bench_skinny.py > gpurun_out/r03b_skinny.log 2>&1 || { tail -30 gpurun_out/r03b_skinny.log; exit 1; }
cat gpurun_out/r03b_skinny.log
timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests --deselect "tests/test_gpu_dit.py::test_apg_euler_multichunk" > gpurun_out/r03b_all.log 2>&1; echo "pytest rc=$?"; tail -5 gpurun_out/r03b_all.log
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03b_bench.json 2> gpurun_out/r03b_bench.err || { tail -30 gpurun_out/r03b_bench.err; exit 1; }
cat gpurun_out/r03b_bench.json
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --seconds 10 --infer-steps 8 --turbo > gpurun_out/r03b_turbo.json 2> gpurun_out/r03b_turbo.err || { tail -30 gpurun_out/r03b_turbo.err; exit 1; }
cat gpurun_out/r03b_turbo.json
rm -rf gpurun_out/probe
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d gpurun_out/probe -o run -- python3 tools/prof_dit.py --seconds 20 --forwards 1 > gpurun_out/probe.log 2>&1 || { tail -20 gpurun_out/probe.log; exit 1; }
python3 tools/rocpd_schema.py $(find gpurun_out/probe -name "*.db" | head -1) > gpurun_out/r03b_schema.txt 2>&1
rm -rf gpurun_out/probe
echo done
