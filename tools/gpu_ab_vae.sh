set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_vae.py tests/test_gpu_long.py -k "vae or decode or encode or resunit or conv" -m gpu > gpurun_out/ru_tests.log 2>&1
rc=$?; tail -5 gpurun_out/ru_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/ab_vae.py tools/ab/libacehip_ref.so > gpurun_out/ab_vae.txt 2>&1; tail -1 gpurun_out/ab_vae.txt
