#!/bin/bash
# Round 6: per-level HBM traffic of configs[1]'s wave (FETCH_SIZE, WRITE_SIZE, L2 hit/miss per k_level dispatch)
# beside the engine's own per-level statistics (FGI_TRACE=1: frontier, edges, pull candidates and probes)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/r14u
FGI_TRACE=1 timeout -k 10 200 python profiles/wave_levels.py rmat24 > gpurun_out/r14u/trace.log 2>&1 || { echo "trace rc=$?"; exit 1; }
PMC_PASSES="FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum" bash profiles/pmc_levels.sh r14u rmat24 || { echo "pmc rc=$?"; exit 1; }
python3 profiles/pmc_levels.py gpurun_out/pmcl_r14u > gpurun_out/r14u/levels.txt
echo done
