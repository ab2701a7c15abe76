#!/bin/bash
# Collects the rocprofv3 evidence for bench.py on the GPU box (run from the repo root):
#   1. kernel trace + stats (per-kernel average durations: compare with bench.py's roofline)
#   2. separate PMC passes (one counter group per pass, as MI355X_MICROARCH.md prescribes):
#      FETCH_SIZE | WRITE_SIZE | TCC_HIT_sum,TCC_MISS_sum | TCC_EA0_ATOMIC_sum
# Output: gpurun_out/prof_<tag>/...  Usage: profiles/run_profile.sh <tag> [bench args...]
set -o pipefail
TAG=${1:-r01}
shift
ARGS=${@:-"--steps 5 --warmup 1 --no-cpu"}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T -d "$OUT/trace" -o run --output-format csv -- \
    python3 "$R/bench.py" $ARGS > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err" || exit 11
for pmc in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" TCC_EA0_ATOMIC_sum; do
    name=$(echo "$pmc" | tr ' ' '_')
    timeout -k 10 300 rocprofv3 --pmc $pmc -T -d "$OUT/pmc_$name" -o run --output-format csv -- \
        python3 "$R/bench.py" $ARGS > "$OUT/pmc_${name}_bench.json" 2> "$OUT/pmc_${name}.err" || exit 12
done
echo "profile $TAG done"
