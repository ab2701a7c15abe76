#!/bin/bash
# Kernel trace of bench_configs.py (e.g. --only churn): per-kernel durations.
# Usage: profiles/trace_configs.sh <tag> <bench_configs args...>
TAG=${1:-c}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/trace_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$R/bench_configs.py" "$@" > "$OUT/out.jsonl" 2> "$OUT/out.err"
rc=$?
[ -s "$OUT/trace/run_kernel_trace.csv" ] || exit $rc
exit 0
