#!/bin/bash
# Kernel trace of the streaming mix in batch mode (bench_configs.py --only stream): per-kernel
# durations of one round's submission. Usage: profiles/trace_stream.sh <tag> [rounds]
TAG=${1:-s}
ROUNDS=${2:-10}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/trace_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$R/bench_configs.py" --only stream --no-cpu --rounds "$ROUNDS" > "$OUT/stream.jsonl" 2> "$OUT/stream.err"
rc=$?
# the kernel trace is complete once the tool has written its files (an exit fault after that is
# the profiler's own teardown)
[ -s "$OUT/trace/run_kernel_trace.csv" ] || exit $rc
exit 0
