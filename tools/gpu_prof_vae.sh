set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rm -rf gpurun_out/pvae
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pvae -o run -- python3 tools/prof_dit.py --forwards 0 --vae > gpurun_out/pvae.log 2>&1 && python3 tools/rocprof_summary.py $(find gpurun_out/pvae -name "*.db" | head -1) > gpurun_out/vae_kernel_stats.md; rc=$?
find gpurun_out/pvae -name "*kernel_stats*" -exec cp {} gpurun_out/vae_kstats.csv \; ; rm -rf gpurun_out/pvae; exit $rc
