#!/bin/bash
# Kernel trace of a short bench run (no PMC): per-dispatch timeline for gap analysis.
# Usage: profiles/trace_only.sh <tag> [bench args]
TAG=${1:-t}; shift
ARGS=${@:-"--steps 5 --warmup 1 --no-cpu"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/trace_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$R/bench.py" $ARGS > "$OUT/bench.json" 2> "$OUT/bench.err"
