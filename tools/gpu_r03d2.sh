#!/bin/bash
# turbo 10 s song timeline (one timed song after one warmup): where the encoder phase goes
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rm -rf gpurun_out/tl
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl -o run -- python3 bench.py --turbo --seconds 10 --infer-steps 8 --steps 1 --warmup 1 --no-cpu-baseline --no-config1 > gpurun_out/r03d_tl_bench.json 2> gpurun_out/r03d_tl.err || { tail -20 gpurun_out/r03d_tl.err; exit 1; }
DB=$(find gpurun_out/tl -name "*.db" | head -1)
# the 3rd song's start: the text encoder's first kernel after two songs (warmup + timed) ...
python3 tools/timeline.py $DB --mark wav_peak --nth 1 --count 3600 > gpurun_out/r03d_timeline_all.txt
rm -rf gpurun_out/tl
grep -n "embed\|gemv_small" gpurun_out/r03d_timeline_all.txt | head -20
tail -45 gpurun_out/r03d_timeline_all.txt
