set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t2.log 2>&1; rc=$?; tail -5 gpurun_out/t2.log; [ $rc = 0 ] || exit $rc
[ -n "$MICRO" ] && { for m in $MICRO; do timeout -k 10 200 python tools/$m || exit 1; done; }
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench2.json 2> gpurun_out/bench2.err && cat gpurun_out/bench2.json
