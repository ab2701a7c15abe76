#!/bin/bash
# PMC passes over bench_configs.py --only churn (configs[3]); k_prune_rows rows of each pass.
# Usage (repo root, GPU box): profiles/pmc_prune.sh <tag>
TAG=${1:-p}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmcp_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
for pmc in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $pmc -T -d "$OUT/p$i" -o run --output-format csv -- \
        python3 "$R/bench_configs.py" --only churn --no-cpu --steps 2 > "$OUT/p$i.out" 2> "$OUT/p$i.err"
    [ -n "$(find "$OUT/p$i" -name '*counter_collection.csv' 2>/dev/null)" ] || exit 30
done
echo "pmc passes done"
