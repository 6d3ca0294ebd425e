#!/bin/bash
# The other BASELINE configs on one box (600 s / 60 steps, repaint, turbo 10 s, base 10 s) and a
# kernel trace of the turbo song.  Every GPU step under its own timeout; a failure ends the script.
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r04c}
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --seconds 600 --infer-steps 60 > gpurun_out/${TAG}_bench_600s.json 2> gpurun_out/${TAG}_b600.err || { tail -20 gpurun_out/${TAG}_b600.err; exit 1; }
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --repaint > gpurun_out/${TAG}_bench_repaint.json 2> gpurun_out/${TAG}_brp.err || { tail -20 gpurun_out/${TAG}_brp.err; exit 1; }
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --turbo --seconds 10 --infer-steps 8 > gpurun_out/${TAG}_bench_turbo10s.json 2> gpurun_out/${TAG}_btu.err || { tail -20 gpurun_out/${TAG}_btu.err; exit 1; }
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --seconds 10 > gpurun_out/${TAG}_bench_base10s.json 2> gpurun_out/${TAG}_bb10.err || { tail -20 gpurun_out/${TAG}_bb10.err; exit 1; }
for f in 600s repaint turbo10s base10s; do python -c "import json; d=json.load(open('gpurun_out/${TAG}_bench_$f.json')); print('$f', d['value'], d['dit_ms_per_step'], d['vae_ms_per_song'], d['roofline']['achieved'])"; done
rm -rf gpurun_out/tprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/tprof -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --turbo --seconds 10 --infer-steps 8 > gpurun_out/${TAG}_turbo_prof.json 2> gpurun_out/${TAG}_turbo_prof.err || { tail -20 gpurun_out/${TAG}_turbo_prof.err; exit 1; }
python3 tools/rocprof_summary.py $(find gpurun_out/tprof -name "*.db" | head -1) > gpurun_out/${TAG}_turbo10s_kernel_stats.md
rc=$?
rm -rf gpurun_out/tprof
head -25 gpurun_out/${TAG}_turbo10s_kernel_stats.md
exit $rc
