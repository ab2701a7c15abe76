#!/bin/bash
# Per-dispatch PMC passes over profiles/wave_levels.py (3 configs[1] waves), one counter group per
# pass (MI355X_MICROARCH.md: separate --pmc passes; 2 x FETCH_SIZE + WRITE_SIZE for HBM bytes on
# gfx950). Output gpurun_out/pmcl_<tag>/<pass>/...; summarise with profiles/pmc_levels.py.
# Usage (repo root, GPU box): profiles/pmc_levels.sh <tag> [workload, default rmat24]
TAG=${1:-l}
CFG=${2:-rmat24}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmcl_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
i=0
# PMC_PASSES="A B;C D" replaces the default counter groups (one pass per ';'-separated group)
if [ -n "${PMC_PASSES:-}" ]; then IFS=';' read -r -a passes <<< "$PMC_PASSES"; else passes=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_ATOMIC_sum"); fi
for pmc in "${passes[@]}"; do
    i=$((i+1))
    timeout -s KILL 150 rocprofv3 --pmc $pmc -T -d "$OUT/p$i" -o run --output-format csv -- \
        python3 "$R/profiles/wave_levels.py" "$CFG" > "$OUT/p$i.out" 2> "$OUT/p$i.err" || exit 30
done
echo "pmc passes done"
