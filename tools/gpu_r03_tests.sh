#!/bin/bash
# full GPU suite + smoke on the current tree
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r03zz}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_gpu_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
