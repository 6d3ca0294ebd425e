#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rm -rf gpurun_out/kt
VARIANTS=8 SHAPES=eq_k6144,down,qkv,o,swiglu COLD=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt -o run -- python3 tools/bench_gemm.py > gpurun_out/r03j.log 2>&1 || { tail -20 gpurun_out/r03j.log; exit 1; }
python3 tools/rocprof_summary.py $(find gpurun_out/kt -name "*.db" | head -1) > gpurun_out/r03j_stats.md 2>&1
python3 - <<'PY' > gpurun_out/r03j_names.txt
import sqlite3,glob
db=glob.glob('gpurun_out/kt/**/*.db',recursive=True)[0]
cur=sqlite3.connect(db).cursor()
for n,c,a in cur.execute("select name,count(*),avg(duration) from kernels group by name order by sum(duration) desc limit 20"):
    print(c, round(a/1e3,1), n[:400])
PY
cat gpurun_out/r03j_names.txt
rm -rf gpurun_out/kt
