#!/bin/bash
# Round-4 evidence on one GPU box: the whole -m gpu suite, the three counter passes of the
# roofline kernel (tools/pmc_roofline.py), the default bench line with those counters
# spliced in (labelled), and the kernel-trace stats of the same bench command.
# Every GPU step under its own timeout; a failure ends the script.
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r04z}
lscpu | grep -E "Model name|^CPU\(s\)" > gpurun_out/${TAG}_host.txt
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
if [ "$SKIP_TESTS" != 1 ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_gpu_tests.log
[ $rc -ne 0 ] && exit $rc
fi
rm -rf gpurun_out/pmc_f gpurun_out/pmc_w gpurun_out/pmc_s gpurun_out/prof
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_f -o run -- python3 tools/prof_dit.py --forwards 1 > gpurun_out/pmc_f.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_w -o run -- python3 tools/prof_dit.py --forwards 1 > gpurun_out/pmc_w.log 2>&1 && \
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES --kernel-trace -d gpurun_out/pmc_s -o run -- python3 tools/prof_dit.py --forwards 1 > gpurun_out/pmc_s.log 2>&1 && \
python3 tools/pmc_roofline.py $(find gpurun_out/pmc_f -name "*.db" | head -1) $(find gpurun_out/pmc_w -name "*.db" | head -1) \
    $(find gpurun_out/pmc_s -name "*.db" | head -1) gpurun_out/${TAG}_pmc_roofline.json --M 6000 --calls 24 \
    --box "$(hostname)" --git "${GIT_HEAD:-unknown}" > gpurun_out/${TAG}_pmc_roofline.txt 2>&1
rc=$?; cat gpurun_out/${TAG}_pmc_roofline.txt | head -40
rm -rf gpurun_out/pmc_f gpurun_out/pmc_w gpurun_out/pmc_s
[ $rc -ne 0 ] && { tail -20 gpurun_out/pmc_s.log; exit $rc; }
timeout -k 10 600 python bench.py --pmc-json gpurun_out/${TAG}_pmc_roofline.json > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { tail -30 gpurun_out/${TAG}_bench.err; exit 1; }
cat gpurun_out/${TAG}_bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.err || { tail -20 gpurun_out/${TAG}_prof.err; exit 1; }
python3 tools/rocprof_summary.py $(find gpurun_out/prof -name "*.db" | head -1) > gpurun_out/${TAG}_kernel_stats.md
rc=$?
rm -rf gpurun_out/prof
exit $rc
