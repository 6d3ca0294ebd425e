#!/bin/bash
# end-of-round-3 evidence: full GPU suite + smoke, counter passes, default bench line, kernel
# stats, then the other configs' lines.  Every GPU step under its own timeout.
set -o pipefail
mkdir -p gpurun_out
TAG=${TAG:-r03z}
bash tools/gpu_r03_round.sh || exit $?
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -1 gpurun_out/${TAG}_smoke.log
SKIP_TESTS2=1 TAG=$TAG bash tools/gpu_r03c2.sh
