set -o pipefail
mkdir -p gpurun_out
MODES=1,2,3,4,0 timeout -k 10 200 python tools/ab_tailsplit.py
