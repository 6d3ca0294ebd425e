set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1 || { tail -30 gpurun_out/t.log; exit 1; }
tail -1 gpurun_out/t.log
for m in 1 0 1 0; do ACEHIP_FUSE_ROWADD=$m timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail -20 gpurun_out/ab.err; exit 1; }; python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('rowadd=$m', d['value'], d['dit_ms_per_step'])"; done
