#!/bin/bash
# One parametrised GPU-box runner (replaces the per-experiment gpu_r0*.sh one-liners).
#
# usage (inside gpurun):  tools/gpu_run.sh TAG STEP [STEP ...]
#
# Each STEP runs under its own time limit, writes gpurun_out/<TAG>_<name>.log, and the chain
# stops at the first failure (no GPU step runs after a fault, abort or time-out).  Steps:
#   tests[=pytest -k expr]     pytest -m gpu (one process, per-test 120 s thread timeout)
#   smoke                      __graft_entry__.smoke()
#   bench[=bench.py args]      bench.py (default: --steps 2 --warmup 1), JSON line to <TAG>_bench.json
#   stats[=bench.py args]      rocprofv3 --kernel-trace --stats of a bench run → gpurun_out/<TAG>_stats/
#   pmc=COUNTERS[=bench args]  one rocprofv3 --pmc pass (counters space-separated) → gpurun_out/<TAG>_pmc_N/
#   py=SCRIPT[=args]           python -u SCRIPT args (A/B tools, micro-benchmarks)
#   pystats=SCRIPT[=args]      rocprofv3 --kernel-trace --stats of a python script → gpurun_out/<TAG>_pystats_N/
#   pypmc=COUNTERS=SCRIPT[=args]  one --pmc pass over a python script → gpurun_out/<TAG>_pypmc_N/
#   env=VAR=VAL                export VAR=VAL for the following steps
set -o pipefail
TAG=${1:?tag}; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
n_pmc=0
n_py=1
run() {  # name seconds cmd...
    local name=$1 secs=$2; shift 2
    local log=gpurun_out/${TAG}_${name}.log
    echo "== $name ($secs s): $*"
    timeout -k 10 "$secs" "$@" > "$log" 2>&1
    local rc=$?
    tail -5 "$log"
    if [ $rc -ne 0 ]; then echo "== $name failed rc=$rc (see $log)"; exit $rc; fi
}
summarize() {  # trace dir → markdown kernel table; the trace database itself is dropped (gpurun_out ≤ 64 MiB)
    local db
    db=$(find "$1" -name "*.db" | head -1)
    [ -n "$db" ] && python3 tools/rocprof_summary.py "$db" > "$2" && rm -rf "$1"
}
for step in "$@"; do
    kind=${step%%=*}; arg=""
    [ "$kind" != "$step" ] && arg=${step#*=}
    case "$kind" in
        tests)
            if [ -n "$arg" ]; then
                run tests_sel 1100 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "$arg"
            else
                run tests 1100 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
            fi ;;
        smoke)
            run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
        bench)
            run bench 600 python -u bench.py ${arg:---steps 2 --warmup 1}
            grep '^{' gpurun_out/${TAG}_bench.log | tail -1 > gpurun_out/${TAG}_bench.json ;;
        stats)
            run stats 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_stats -o run -- \
                python3 bench.py ${arg:---steps 1 --warmup 1 --no-cpu-baseline}
            summarize gpurun_out/${TAG}_stats gpurun_out/${TAG}_kernel_stats.md ;;
        pmc)
            counters=${arg%%=*}; bargs=""
            [ "$counters" != "$arg" ] && bargs=${arg#*=}
            n_pmc=$((n_pmc + 1))
            run pmc_$n_pmc 240 rocprofv3 --pmc $counters -d gpurun_out/${TAG}_pmc_$n_pmc -o run -- \
                python3 bench.py ${bargs:---steps 1 --warmup 0 --no-cpu-baseline} ;;
        py)
            script=${arg%%=*}; pargs=""
            [ "$script" != "$arg" ] && pargs=${arg#*=}
            name=$(basename "$script" .py)
            [ -e "gpurun_out/${TAG}_${name}.log" ] && name="${name}_$((++n_py))"
            run "$name" 900 python -u "$script" $pargs ;;
        pystats)
            script=${arg%%=*}; pargs=""
            [ "$script" != "$arg" ] && pargs=${arg#*=}
            n_pmc=$((n_pmc + 1))
            run pystats_$n_pmc 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_pystats_$n_pmc -o run -- \
                python3 "$script" $pargs
            summarize gpurun_out/${TAG}_pystats_$n_pmc gpurun_out/${TAG}_pystats_${n_pmc}_kernel_stats.md ;;
        pypmc)
            counters=${arg%%=*}; rest=${arg#*=}
            script=${rest%%=*}; pargs=""
            [ "$script" != "$rest" ] && pargs=${rest#*=}
            n_pmc=$((n_pmc + 1))
            run pypmc_$n_pmc 240 rocprofv3 --pmc $counters --kernel-trace -d gpurun_out/${TAG}_pypmc_$n_pmc -o run -- \
                python3 "$script" $pargs ;;
        env)
            export "$arg"; echo "== env $arg" ;;
        *)
            echo "unknown step: $step"; exit 2 ;;
    esac
done
