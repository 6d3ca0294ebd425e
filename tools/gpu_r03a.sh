#!/bin/bash
# round 3, first box: changed GPU tests first, then the whole GPU suite, a quick bench
# line, and a schema probe of a short counter pass (same-pass durations for the clock).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu \
  tests/test_gpu_condenc.py::test_fsq_bit_exact_exhaustive tests/test_vae.py tests/test_gpu_integration.py \
  "tests/test_gpu_dit.py::test_apg_euler_multichunk" > gpurun_out/r03a_new.log 2>&1 || { tail -40 gpurun_out/r03a_new.log; exit 1; }
tail -3 gpurun_out/r03a_new.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu tests > gpurun_out/r03a_all.log 2>&1 || { tail -40 gpurun_out/r03a_all.log; exit 1; }
tail -3 gpurun_out/r03a_all.log
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/r03a_bench.json 2> gpurun_out/r03a_bench.err || { tail -30 gpurun_out/r03a_bench.err; exit 1; }
cat gpurun_out/r03a_bench.json
rm -rf gpurun_out/probe
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace -d gpurun_out/probe -o run -- python3 tools/prof_dit.py --seconds 20 --forwards 1 > gpurun_out/probe.log 2>&1 || { tail -20 gpurun_out/probe.log; exit 1; }
python3 tools/rocpd_schema.py $(find gpurun_out/probe -name "*.db" | head -1) > gpurun_out/r03a_schema.txt 2>&1
rm -rf gpurun_out/probe
echo done
