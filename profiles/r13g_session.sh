#!/bin/bash
# Round 5: why configs[1]'s level 0 gathers its pool entries ~6x slower than level 4 — per-dispatch TLB,
# L2-request latency and instruction-cache counters of the wave's kernels (profiles/pmc_levels.sh)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/r13g; mkdir -p $out
cd $R
PMC_PASSES="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_REQUEST_sum TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum;TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum;SQC_ICACHE_MISSES SQC_ICACHE_HITS;TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum" \
  bash profiles/pmc_levels.sh r13g rmat24 > $out/pmc.log 2>&1 || { echo "pmc rc=$?"; tail -5 $out/pmc.log; exit 1; }
python3 profiles/pmc_levels.py gpurun_out/pmcl_r13g > $out/pmc_levels.txt 2>&1 || true
cat $out/pmc_levels.txt
