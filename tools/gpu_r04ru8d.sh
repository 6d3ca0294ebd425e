#!/bin/bash
# (historical: the RU8_D / RU8_PIPE variants were removed after this A/B)
# ru8 W ring distance 2 (tree) vs 3 (libacehip_d3.so) vs 3 + the pipelined K loop
# (libacehip_d3p.so), all on ACEHIP_RU7=2: 240 s decode A/B in one process (bit-equality
# reported), then the ru7 / ru8 knob A/B on the tree library
set -o pipefail
mkdir -p gpurun_out
ACEHIP_RU7=2 timeout -k 10 300 python -u tools/ab_vae.py tools/ab/libacehip_d3.so tools/ab/libacehip_d3p.so > gpurun_out/r04ru8d_ab.log 2>&1
rc=$?; tail -2 gpurun_out/r04ru8d_ab.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u tools/ab_env_vae.py 'ACEHIP_RU7=1' 'ACEHIP_RU7=2' > gpurun_out/r04ru8d_ab_env.log 2>&1
rc=$?; tail -3 gpurun_out/r04ru8d_ab_env.log; exit $rc
