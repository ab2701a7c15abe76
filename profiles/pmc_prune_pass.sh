#!/bin/bash
# ONE PMC pass over bench_configs.py --only churn (configs[3]); its cooperative prune launch makes
# rocprofv3 crash at process exit after the counters are written, so each pass is the last GPU step
# of its own gpurun call. Usage (repo root, GPU box): profiles/pmc_prune_pass.sh <tag> <counter>
TAG=${1:-p}; PMC=${2:-FETCH_SIZE}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmcp_$TAG/$PMC
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc $PMC -T -d "$OUT" -o run --output-format csv -- \
    python3 "$R/bench_configs.py" --only churn --no-cpu --steps 2 > "$OUT/out.jsonl" 2> "$OUT/err.log"
rc=$?
echo "rocprofv3 rc=$rc"
find "$OUT" -name '*counter_collection.csv' | head -1
exit $rc
